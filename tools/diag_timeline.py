#!/usr/bin/env python3
"""Diagnostic (not product): per-wave, per-step timeline of one specialised-decoder iteration from a diagnostic
library (make -C srsran_projectvtlmo_amd/csrc diag: libsrsran_ldpc_hip_diagfull.so stamps every phase,
libsrsran_ldpc_hip_diag.so only step start and barrier exit), block 0 of a 128-CB batch, last iteration.

Stamps per (step S, wave w) (s_memtime, ~1 tick per shader clock): 0 step start, 1 soft reads landed, 2 pass 1 done,
3 row scale done, 4 writes drained (the wave is at the barrier), 5 after the barrier. A wave that has no role in a step
(its group idle, or its row beyond the adaptive layer count) writes only 0, 4 and 5.

Apportioning the barrier parking (SQ_WAIT_ANY in the PMC passes), per step:
  work(w)  = stamp4 - stamp0       the wave's own path through the step (role code, LDS latency, drain)
  park(w)  = stamp5 - stamp4       waiting at the barrier for the last wave
  crit     = max_w work(w)         the step's critical path: no wave can leave before it
and over waves: park of waves without a role ("idle"), of role waves in the group whose longest wave is shorter than
the other group's ("role imbalance": two-row steps and pipelined chains), and of role waves within the critical group
("spread": the same code on different lanes / SIMD contention). The critical wave parks for ~0 ticks: its work is the
step's true dependency chain.

usage: python tools/diag_timeline.py BG Z [iters] [diagfull|diag] [unit letter for non-core graphs]"""
import collections
import ctypes
import sys
from pathlib import Path

import torch  # noqa: F401

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
bg, Z = int(sys.argv[1]), int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8
variant = sys.argv[4] if len(sys.argv) > 4 else "diagfull"
unit = sys.argv[5] if len(sys.argv) > 5 else None
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{variant}.so"
L = _lib.load()
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
print(f"{variant} kernel {ev0.elapsed_time(ev1) * 1e3:.1f} us (BG{bg} Z={Z}, {iters} it, {n} CBs)")
fn = getattr(L, "ldpc_hip_diag2_read" + (f"_{unit}" if unit else ""))
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
N2 = 64 * 16 * 8
b = (ctypes.c_uint64 * N2)()
assert fn(b, N2) == 0


def st(S, w, k):
    return b[(S * 16 + w) * 8 + k]


nsteps = next(S for S in range(64) if st(S, 0, 0) == 0 and st(S, 0, 5) == 0)
nw = max(w + 1 for w in range(16) if st(0, w, 0) != 0)
full = variant == "diagfull"
print(f"{nsteps} steps, {nw} waves; ticks per step: span, critical work, per-wave work (* = no role) and parking")
tot = collections.Counter()
for S in range(nsteps):
    t0 = min(st(S, w, 0) for w in range(nw))
    end = max(st(S, w, 5) for w in range(nw))
    work, park, role = {}, {}, {}
    for w in range(nw):
        a, d, e = st(S, w, 0), st(S, w, 4) if full else st(S, w, 5), st(S, w, 5)
        role[w] = (not full) or (st(S, w, 1) >= a and st(S, w, 1) - a < 10**6)
        work[w] = d - a
        park[w] = e - d
    crit = max(work[w] for w in range(nw) if role[w]) if any(role.values()) else 0
    tot["span"] += end - t0
    tot["crit"] += crit
    if full:
        half = nw // 2
        grp = [[w for w in range(nw) if role[w] and (w < half) == (k == 0)] for k in (0, 1)]
        gmax = [max((work[w] for w in gg), default=0) for gg in grp]
        for w in range(nw):
            if not role[w]:
                tot["park_idle"] += park[w]
            else:
                k = 0 if w < half else 1
                if gmax[k] < max(gmax):
                    tot["park_role_imbalance"] += park[w]
                else:
                    tot["park_spread"] += park[w]
    cells = " ".join(f"{work[w]:5d}{'' if role[w] else '*'}/{park[w]:<4d}" for w in range(nw))
    print(f"{S:2d} span {end - t0:5d} crit {crit:5d} | {cells}")
print("iteration totals (ticks):", dict(tot))
if full:
    allpark = tot["park_idle"] + tot["park_role_imbalance"] + tot["park_spread"]
    print(f"parking over waves: {allpark} = idle {tot['park_idle']} + role imbalance {tot['park_role_imbalance']} "
          f"+ spread {tot['park_spread']}; critical chain {tot['crit']} of {tot['span']} span ticks")
