#!/usr/bin/env python3
"""Generates the committed golden fixtures (tests/golden/*.npz) with the CPU oracle (oracle/ldpc_oracle.c).

These are regression fixtures of the oracle, not reference outputs: the reference's own .dat vectors are absent
from the snapshot and building or running the reference is denied. The oracle itself is pinned by
tests/test_oracle.py (the reference's in-source known-answer tests + round-trip properties).

Contents:
  c1.npz  BG2 Z=52, 1 CB, 6 iterations: message 504 random bits (seed 0) + CRC16 -> 520-bit message -> encoded
          2,600 bits -> LLR +-10; decoded without CRC (ldpc_enc_dec_test.cpp procedure) and with CRC16 early stop;
          plus the length sweep create_range(12Z, 50Z, 3) at 1 iteration.
  c2.npz  BG1 Z=384, 4 CBs of the C2 benchmark distribution (+-10, seeded), 8 iterations, no CRC.
  c3.npz  BG2 Z=208, 8 CBs: 2,056 random bits + CRC24B, BPSK 2.0 + N(0,1) quantised (seed 2), 10 iterations, CRC24B
          early stop (iteration counts recorded).
"""
from pathlib import Path
import sys

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent


def bits_of(v, n):
    return np.array([(v >> (n - 1 - i)) & 1 for i in range(n)], dtype=np.uint8)


def c1():
    rng = np.random.default_rng(0)
    Z, K = 52, 10
    data = rng.integers(0, 2, K * Z - 16).astype(np.uint8)
    msg = np.concatenate([data, bits_of(O.crc_bits(O.CRC16, data), 16)])
    cw = O.ldpc_encode(2, Z, msg)
    llr = np.where(cw == 1, -10, 10).astype(np.int8)
    out_nocrc, _ = O.ldpc_decode(2, Z, llr, 6)
    out_crc, it = O.ldpc_decode(2, Z, llr, 6, crc_poly=O.CRC16)
    sweep_len = [12 * Z, 12 * Z + (50 * Z - 12 * Z) // 2, 50 * Z]
    sweep_out = np.stack([O.ldpc_decode(2, Z, llr[:L], 1)[0] for L in sweep_len])
    np.savez(OUT / "c1.npz", msg=msg, llr=llr, out_nocrc=out_nocrc, out_crc=out_crc, iters_crc=np.int32(it),
             sweep_len=np.array(sweep_len, np.int32), sweep_out=sweep_out)


def c2():
    rng = np.random.default_rng(0)
    llr = (rng.integers(0, 2, (4, 66 * 384)) * 20 - 10).astype(np.int8)
    out = np.stack([O.ldpc_decode(1, 384, l, 8)[0] for l in llr])
    np.savez(OUT / "c2.npz", llr=llr, out=out)


def c3():
    rng = np.random.default_rng(2)
    Z = 208
    llrs, outs, its = [], [], []
    for _ in range(8):
        data = rng.integers(0, 2, 10 * Z - 24).astype(np.uint8)
        msg = np.concatenate([data, bits_of(O.crc_bits(O.CRC24B, data), 24)])
        cw = O.ldpc_encode(2, Z, msg)
        x = np.where(cw == 1, -2.0, 2.0).astype(np.float32) + rng.standard_normal(cw.size).astype(np.float32)
        llr = O.quantize_array(x, 8.0)
        out, it = O.ldpc_decode(2, Z, llr, 10, crc_poly=O.CRC24B)
        llrs.append(llr)
        outs.append(out)
        its.append(0 if it is None else it)
    np.savez(OUT / "c3.npz", llr=np.stack(llrs), out=np.stack(outs), iters=np.array(its, np.int32))


if __name__ == "__main__":
    c1()
    c2()
    c3()
    print("golden fixtures written to", OUT)
