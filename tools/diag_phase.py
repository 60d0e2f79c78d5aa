#!/usr/bin/env python3
"""Diagnostic (not product): phase timeline of every wave in every step (block 0, last iteration) from the
LDPC_HIP_DIAG_PHASE build (make -C srsran_projectvtlmo_amd/csrc exp NAME=phase FLAGS=-DLDPC_HIP_DIAG_PHASE).

Phases (s_memtime, relative to the earliest step start): 7 step start, 0 row entry, 1 addresses done, 2 pass 1 done,
3 merge + scaling done, 4 pass 2 issued, 5 LDS drained, 6 after barrier."""
import ctypes
import sys
from pathlib import Path

import torch  # noqa: F401

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / "libsrsran_ldpc_hip_phase.so"
L = _lib.load()
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402

n, iters = 128, 8
bg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
Z = int(sys.argv[2]) if len(sys.argv) > 2 else 384
ctx = _lib.Context(0)
specs, ls, os_ = cc.uniform_batch_specs(n, bg, Z, iters)
plan = cc.DecodePlan(ctx, specs)
g = torch.Generator(device="cuda").manual_seed(1)
llr = (torch.randint(0, 2, (n, ls), device="cuda", dtype=torch.int8, generator=g) * 20 - 10).to(torch.int8)
out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
for _ in range(3):
    plan.launch(llr.data_ptr(), out.data_ptr(), 0, 0)
torch.cuda.synchronize()
L.ldpc_hip_diag2_read.restype = ctypes.c_int
L.ldpc_hip_diag2_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
b = (ctypes.c_uint64 * (64 * 16 * 8))()
L.ldpc_hip_diag2_read(b, 64 * 16 * 8)
nw = 16
steps = cc.schedule_groups(bg, Z) + 8  # steps with stamps (a wide group may take more than one step)
tot = {k: 0 for k in ("addr", "pass1", "merge", "pass2", "drain", "barrier", "head")}
for s in range(steps):
    rows = []
    vals = [b[(s * 16 + w) * 8 + 7] for w in range(nw) if b[(s * 16 + w) * 8 + 7] != 0]
    if not vals:
        break
    base = min(vals)
    for w in range(nw):
        p = [b[(s * 16 + w) * 8 + q] for q in range(8)]
        if p[7] == 0:
            continue
        if p[0] == 0:
            rows.append(f"w{w:2d} idle  drain {p[5] - base:5d} bar {p[6] - base:5d}")
            continue
        rows.append(f"w{w:2d} start {p[7] - base:5d} row {p[0] - base:5d} addr {p[1] - base:5d} p1 {p[2] - base:5d} "
                    f"mg {p[3] - base:5d} p2 {p[4] - base:5d} drain {p[5] - base:5d} bar {p[6] - base:5d}")
    print(f"--- step {s}")
    print("\n".join(rows))
