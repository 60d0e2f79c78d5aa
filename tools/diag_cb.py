#!/usr/bin/env python3
"""Diagnostic (not product): where a codeblock's time goes outside the iterations. LDPC_HIP_DIAG_CB build
(s_memrealtime, 100 MHz, per workgroup): 0 entry, 1 prologue done (soft bits and tables in LDS, after the barrier),
2 lanes and masks ready (first iteration starts), 3 iterations done, 4 hard decision and CRC done, 5 output and result
stored. BG1 Z=384, 6 layers (C4's UE0 rate), one iteration, 512 CBs (two rounds of one CB per CU).

usage: python tools/diag_cb.py [lib suffix, default diagcb] [n CBs] [iterations] [layers: 6 | full | c3]
  c3: BG2 Z=208, all-zero codeword (+10 LLRs, every CB passes its CRC24B after one iteration), early stop"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{sys.argv[1] if len(sys.argv) > 1 else 'diagcb'}.so"
L = _lib.load()
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1
mode = sys.argv[4] if len(sys.argv) > 4 else "6"
bg, Z = (2, 208) if mode == "c3" else (1, 384)
nz = {"full": 66 * 384, "c3": 50 * 208}.get(mode, 9728)
ctx = _lib.Context(0)
specs, ls, os_ = cc.uniform_batch_specs(n, bg, Z, iters, crc_mode=_lib.CRC_MODE_EARLY_STOP if mode == "c3" else 0,
                                        crc_poly=_lib.CRC24B if mode == "c3" else -1)
plan = cc.DecodePlan(ctx, specs)
g = torch.Generator(device="cuda").manual_seed(1)
llr = torch.zeros((n, ls), device="cuda", dtype=torch.int8)
if mode == "c3":
    llr[:, :nz] = 10
else:
    llr[:, :nz] = torch.randint(0, 2, (n, nz), device="cuda", dtype=torch.int8, generator=g) * 20 - 10
out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(4):
    ev0.record(s)
    plan.launch(llr.data_ptr(), out.data_ptr(), 0, s.cuda_stream)
    ev1.record(s)
    torch.cuda.synchronize()
print(f"kernel {ev0.elapsed_time(ev1) * 1e3:.1f} us (BG{bg} Z={Z} {nz} LLRs, {iters} it, {n} CBs, {mode})")
L.ldpc_hip_diag_cb_read.restype = ctypes.c_int
L.ldpc_hip_diag_cb_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
b = (ctypes.c_uint64 * 8192)()
assert L.ldpc_hip_diag_cb_read(ctx.handle, b, 8192) == 0
a = np.array(b, dtype=np.int64).reshape(1024, 8)[:n, :6]
t0 = a[:, 0].min()
us = (a - t0) * 0.01
names = ["entry", "prologue", "lanes", "iterations", "hd+crc", "stored"]
order = np.argsort(us[:, 0])
per = 512 if mode == "c3" else 256  # workgroups resident at once (BG2 Z=208: two per CU)
for half, idx in (("first round", order[: min(n, per)]), ("second round", order[per:])):
    if len(idx) == 0:
        continue
    u = us[idx]
    print(f"{half}: {len(idx)} workgroups, us after the first entry (min / median / max)")
    for k, name in enumerate(names):
        print(f"  {name:10s} {u[:, k].min():6.2f} {np.median(u[:, k]):6.2f} {u[:, k].max():6.2f}")
    d = np.diff(u, axis=1)
    for k in range(5):
        print(f"  {names[k] + '->' + names[k + 1]:22s} {d[:, k].min():6.2f} {np.median(d[:, k]):6.2f} {d[:, k].max():6.2f}")
ctx.close()
