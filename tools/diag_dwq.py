#!/usr/bin/env python3
"""Diagnostic (not product): where a one-codeblock software-route call's time goes on the device work queue path.
LDPC_HIP_DIAG_DWQ + LDPC_HIP_DIAG_CB build (make -C srsran_projectvtlmo_amd/csrc VARIANT=diagdwq
FLAGS="-DLDPC_HIP_DIAG_DWQ -DLDPC_HIP_DIAG_CB"): per completed item the host's entry, submit and done-seen times
(steady clock) and the device's 100 MHz stamps (claim, item copied, body done), plus the workgroup's decoder phase
stamps (entry, prologue, lanes, iterations, hard decision + CRC, stored).

usage: python tools/diag_dwq.py [calls per case]   (LDPC_HIP_DWQ=0: the launch path's body phases)"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{os.environ.get('DIAG_LIB', 'diagdwq')}.so"
L = _lib.load()
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402
import oracle as O  # noqa: E402  (test vectors only)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
L.ldpc_hip_diag_dwq_read.restype = ctypes.c_uint32
L.ldpc_hip_diag_dwq_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
L.ldpc_hip_diag_cb_read.restype = ctypes.c_int
L.ldpc_hip_diag_cb_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]


def codeword(rng, bg, Z, nllr, amp):
    K = O.BG_K[bg] * Z
    msg = rng.integers(0, 2, K).astype(np.uint8)
    c = O.crc_bits(O.CRC24B, msg[:K - 24])
    msg[K - 24:] = [(c >> (23 - i)) & 1 for i in range(24)]
    cw = O.ldpc_encode(bg, Z, msg)[:nllr]
    x = np.where(cw == 1, -amp, amp) + rng.standard_normal(cw.size)
    return O.quantize_array(x.astype(np.float32), 8.0)


ctx = _lib.Context(0)
dec = cc.ldpc_decoder_hip(ctx)
rng = np.random.default_rng(3)
rec_buf = (ctypes.c_uint64 * (8 * 4096))()
cb_buf = (ctypes.c_uint64 * 8192)()
# (name, bg, Z, LLRs): a C4 one-CB TB's BG2 Z=36 codeblock at its full length, and C4's 128-CB TB codeblock (BG1
# Z=384, rate 0.87: 9,728 LLRs, 6 layers)
for name, bg, Z, nllr in (("BG2 Z=36", 2, 36, 50 * 36), ("BG1 Z=384 6 layers", 1, 384, 9728)):
    cfg = cc.configuration()
    cfg.block_conf.tb_common.base_graph = bg
    cfg.block_conf.tb_common.lifting_size = Z
    cfg.algorithm_conf.max_iterations = 8
    crc = cc.crc_calculator("CRC24B")
    llrs = [codeword(rng, bg, Z, nllr, 2.5) for _ in range(8)]
    out = np.zeros(cc.message_bytes(bg, Z), np.uint8)
    full = np.zeros(cc.BG_N_SHORT[bg] * Z, np.int8)
    L.ldpc_hip_diag_dwq_read(rec_buf, 4096)
    phases = []
    its = []
    for k in range(n):
        full[:] = 0
        full[:nllr] = llrs[k % len(llrs)]
        its.append(dec.decode(out, full[:nllr], crc, cfg))
        if k % 10 == 9:
            assert L.ldpc_hip_diag_cb_read(ctx.handle, cb_buf, 8192) == 0
            phases.append(np.array(cb_buf, dtype=np.int64).reshape(1024, 8))
    m = L.ldpc_hip_diag_dwq_read(rec_buf, 4096)
    r = np.array(rec_buf[:8 * m], dtype=np.int64).reshape(m, 8)
    if m == 0:  # LDPC_HIP_DWQ=0: the launch path, one workgroup per call; its phases only
        dd = np.array([np.diff(ph[0, :6]) * 0.01 for ph in phases])
        names = ["prologue", "lanes", "iterations", "hd+crc", "stored"]
        print(f"{name} (launch path): iterations median {np.median([i if i else 0 for i in its]):.0f}; body phases "
              "(us, p50): " + ", ".join(f"{a} {np.median(dd[:, i]):.2f}" for i, a in enumerate(names)))
        continue
    # columns: submit_ns, seen_ns, claim_tick_lo, item_ticks, body_ticks, workgroup, spec + 1, entry_ns
    total = (r[:, 1] - r[:, 7]) / 1e3
    prep = (r[:, 0] - r[:, 7]) / 1e3
    sub_seen = (r[:, 1] - r[:, 0]) / 1e3
    item = r[:, 3] * 0.01
    body = (r[:, 4] - r[:, 3]) * 0.01
    dev = r[:, 4] * 0.01
    print(f"{name}: {m} calls, iterations median {np.median([i if i else 0 for i in its]):.0f}; us, p50 / p10 / p90")
    for lab, v in (("entry -> done seen (host)", total), ("entry -> submitted (host prep)", prep),
                   ("submitted -> done seen", sub_seen), ("device: claim -> item in LDS", item),
                   ("device: body (dematch + decode)", body), ("device: claim -> body done", dev),
                   ("outside the device (pickup + done)", sub_seen - dev)):
        print(f"  {lab:38s} {np.median(v):7.2f} {np.percentile(v, 10):7.2f} {np.percentile(v, 90):7.2f}")
    # the workgroup's body phases for the sampled calls (stamps of the workgroup that ran the call)
    dd = []
    for k, ph in zip(range(9, n, 10), phases):
        wg = int(r[k, 5]) if k < m else None
        if wg is None:
            continue
        st = ph[wg, :6]
        # stamps 6 (body entry) and 7 (the prologue's global loads returned), when the build has them
        extra = [(st[0] - ph[wg, 6]) * 0.01, (ph[wg, 7] - st[0]) * 0.01] if ph[wg, 6] and ph[wg, 7] else [0, 0]
        dd.append(list(np.diff(st) * 0.01) + extra)
    if dd:
        dd = np.array(dd)
        names = ["prologue", "lanes", "iterations", "hd+crc", "stored", "(dematch before it)",
                 "(prologue until its loads returned)"]
        print("  body phases (us, p50): " + ", ".join(f"{a} {np.median(dd[:, i]):.2f}" for i, a in enumerate(names)))
ctx.close()
