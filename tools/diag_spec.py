#!/usr/bin/env python3
"""Diagnostic (not product): per-step, per-wave phase stamps of the specialised decoder (LDPC_HIP_DIAG build) on the
C2 batch. Phases per (step, wave) of block 0, last iteration: 0 step start, 1 soft reads landed, 2 pass 1 done,
3 row scale done, 4 writes drained, 5 after the step barrier.

usage: python tools/diag_spec.py [iters] [lib suffix: diag (stamps 0 and 5 only) | diagfull (all phases)]
"""
import ctypes
import sys
from pathlib import Path

import torch  # noqa: F401

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 8
from srsran_projectvtlmo_amd import _lib  # noqa: E402

variant = sys.argv[2] if len(sys.argv) > 2 else "diag"
_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{variant}.so"
L = _lib.load()
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402

ctx = _lib.Context(0)
n = 128
specs, ls, os_ = cc.uniform_batch_specs(n, 1, 384, iters)
plan = cc.DecodePlan(ctx, specs)
g = torch.Generator(device="cuda").manual_seed(1)
llr = (torch.randint(0, 2, (n, ls), device="cuda", dtype=torch.int8, generator=g) * 20 - 10).to(torch.int8)
out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(3):
    ev0.record(s)
    plan.launch(llr.data_ptr(), out.data_ptr(), 0, s.cuda_stream)
    ev1.record(s)
    torch.cuda.synchronize()
print(f"diag kernel {ev0.elapsed_time(ev1) * 1e3:.1f} us (BG1 Z=384 {iters} it, {n} CBs)")
L.ldpc_hip_diag2_read.restype = ctypes.c_int
L.ldpc_hip_diag2_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
N2 = 64 * 16 * 8
b2 = (ctypes.c_uint64 * N2)()
L.ldpc_hip_diag2_read(b2, N2)
nsteps, nw = 32, 12
tot = 0
print("step | span(start->barrier exit) | per phase, max over waves of (stamp - step start): reads pass1 scale drained barrier")
prev_end = None
for S in range(nsteps):
    st = [b2[(S * 16 + w) * 8 + 0] for w in range(nw)]
    t0 = min(st)
    rows = []
    for k in range(1, 6):
        vals = [b2[(S * 16 + w) * 8 + k] - t0 for w in range(nw) if b2[(S * 16 + w) * 8 + k] >= t0
                and b2[(S * 16 + w) * 8 + k] - t0 < 10**7]
        rows.append(max(vals) if vals else -1)
    gap = (t0 - prev_end) if prev_end else 0
    prev_end = max(b2[(S * 16 + w) * 8 + 5] for w in range(nw))
    tot += prev_end - t0
    print(f"{S:2d} span {prev_end - t0:6d}  reads {rows[0]:5d} pass1 {rows[1]:5d} scale {rows[2]:5d} drained {rows[3]:5d} "
          f"barrier {rows[4]:5d}  start-skew {max(st) - t0:4d}")
print("sum of step spans (ticks):", tot)
