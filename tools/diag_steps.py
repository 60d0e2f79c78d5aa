#!/usr/bin/env python3
"""Diagnostic (not product): per-step cycle stamps of the decoder on the C2 batch, from the LDPC_HIP_DIAG builds.

usage: python tools/diag_steps.py [diag|diagskip] [bg] [Z] [iters]
"""
import ctypes
import sys
from pathlib import Path

import torch  # noqa: F401  (one HIP runtime: torch first)

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

variant = sys.argv[1] if len(sys.argv) > 1 else "diag"
bg = int(sys.argv[2]) if len(sys.argv) > 2 else 1
Z = int(sys.argv[3]) if len(sys.argv) > 3 else 384
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 8

from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{variant}.so"
L = _lib.load()
L.ldpc_hip_diag_read.restype = ctypes.c_int
L.ldpc_hip_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402

ctx = _lib.Context(0)
n = 128
specs, ls, os_ = cc.uniform_batch_specs(n, bg, Z, iters)
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
print(f"{variant}: kernel {ev0.elapsed_time(ev1) * 1e3:.1f} us  (BG{bg} Z={Z} {iters} it, {n} CBs)")
buf = (ctypes.c_uint64 * 4096)()
L.ldpc_hip_diag_read(buf, 4096)
ng = cc.schedule_groups(bg, Z)
stamps = list(buf[: 1 + ng * iters])
d = [stamps[i + 1] - stamps[i] for i in range(len(stamps) - 1)]
tot = stamps[-1] - stamps[0]
print(f"total stamped {tot} s_memtime ticks; per iteration {tot / iters:.0f}; per step {tot / len(d):.0f}")
last = d[(iters - 1) * ng: iters * ng]
print("last-iteration per-step ticks:", last)

L.ldpc_hip_diag2_read.restype = ctypes.c_int
L.ldpc_hip_diag2_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
b2 = (ctypes.c_uint64 * (64 * 16 * 2))()
L.ldpc_hip_diag2_read(b2, 64 * 16 * 2)
nw = 12
print("per step (last iteration): [work ticks per wave] | barrier-exit skew")
for g in range(ng):
    st = [b2[(g * 16 + w) * 2] for w in range(nw)]
    en = [b2[(g * 16 + w) * 2 + 1] for w in range(nw)]
    work = [e - s for s, e in zip(st, en)]
    print(g, "work", work, "start-skew", max(st) - min(st), "end-skew", max(en) - min(en))
