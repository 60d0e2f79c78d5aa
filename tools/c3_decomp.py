#!/usr/bin/env python3
"""Diagnostic (not product): where C3's batch time goes. The C3 input (1024 BG2 Z=208 AWGN codewords, bench.py
extra_c3) decoded with: the C3 settings; 1 and 2 iterations without a CRC; 1 iteration with the CRC checked after;
and the C3 settings on the first 128 / 256 / 512 CBs. Kernel time per batch (HIP events, 20 reps).

usage: python tools/c3_decomp.py [lib.so]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = Path(sys.argv[1]).resolve()
import bench  # noqa: E402
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402
from srsran_projectvtlmo_amd import segmentation as S  # noqa: E402
from srsran_projectvtlmo_amd import synth  # noqa: E402

ctx = _lib.Context(0)
stream = torch.cuda.Stream()
n, bg, z = 1024, 2, 208
rng = np.random.default_rng(2)
msgs = np.zeros((n, 10 * z), np.uint8)
msgs[:, :2056] = rng.integers(0, 2, (n, 2056))
for i in range(n):
    c = S.crc_bits("CRC24B", msgs[i, :2056])
    msgs[i, 2056:] = [(c >> (23 - k)) & 1 for k in range(24)]
llr = synth.codeword_llrs(ctx, bg, z, msgs, 2.0, 1.0, seed=2)


def run(name, cnt, it, mode, poly):
    specs, ls, os_ = cc.uniform_batch_specs(cnt, bg, z, it, None, mode, poly)
    d_llr = torch.zeros((cnt, ls), dtype=torch.int8, device="cuda")
    d_llr[:, : llr.shape[1]] = llr[:cnt]
    d_out = torch.zeros(cnt * os_, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(cnt * 4, dtype=torch.uint8, device="cuda")
    plan = cc.DecodePlan(ctx, specs)
    us = bench._time(lambda: plan.launch(d_llr.data_ptr(), d_out.data_ptr(), d_res.data_ptr(), stream.cuda_stream),
                     stream, 20)
    res = d_res.cpu().numpy().reshape(-1, 4)
    plan.close()
    print(f"{name:34s} CBs {cnt:5d} it {it:2d}  {us:8.1f} us  mean it {res[:, 1].mean():.3f}", flush=True)


run("C3 (ET, 10 it)", 1024, 10, cc.CRC_MODE_EARLY_STOP, cc.CRC24B)
run("no CRC, 1 it", 1024, 1, cc.CRC_MODE_NONE, -1)
run("no CRC, 2 it", 1024, 2, cc.CRC_MODE_NONE, -1)
run("no CRC, 4 it", 1024, 4, cc.CRC_MODE_NONE, -1)
run("ET, 1 it", 1024, 1, cc.CRC_MODE_EARLY_STOP, cc.CRC24B)
for cnt in (128, 256, 512, 768):
    run("C3 (ET, 10 it)", cnt, 10, cc.CRC_MODE_EARLY_STOP, cc.CRC24B)
    run("no CRC, 1 it", cnt, 1, cc.CRC_MODE_NONE, -1)
ctx.close()
