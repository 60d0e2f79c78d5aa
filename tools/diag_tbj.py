#!/usr/bin/env python3
"""Diagnostic (not product): phase stamps of the TB join kernel (LDPC_HIP_DIAG_TBJ build, s_memrealtime, 100 MHz)
in the C4 slot (bench.py extra_c4, last launch). Per workgroup, us after the earliest workgroup's entry:
0 entry, 1 gather + CB flags (after the first barrier), 2 chunk CRC in LDS, 3 arrival counter read, 4 last arriver done.

usage: python tools/diag_tbj.py [lib suffix, default diagtbj]"""
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{sys.argv[1] if len(sys.argv) > 1 else 'diagtbj'}.so"
L = _lib.load()
import bench  # noqa: E402

ctx = _lib.Context(0)
stream = torch.cuda.Stream()
print(bench.extra_c4(ctx, stream, reps=3))
L.ldpc_hip_diag2_read.restype = ctypes.c_int
L.ldpc_hip_diag2_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
b = (ctypes.c_uint64 * (64 * 16 * 8))()
L.ldpc_hip_diag2_read(b, 64 * 16 * 8)
rows = [[b[i * 8 + k] for k in range(5)] for i in range(64)]
rows = [(i, r) for i, r in enumerate(rows) if r[0] != 0]
t0 = min(r[0] for _, r in rows)
print("block  entry  flags  crc  counter  last-done   (us after the first entry)")
for i, r in rows:
    f = ["%6.2f" % ((x - t0) * 0.01) if x >= t0 and x - t0 < 10**6 else "     -" for x in r]
    print(f"{i:5d} " + " ".join(f))
ctx.close()
