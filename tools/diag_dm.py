#!/usr/bin/env python3
"""Diagnostic (not product): phase stamps of the rate dematcher (LDPC_HIP_DIAG_DM build, s_memrealtime, 100 MHz) in
the C4 slot from LLRs (bench.py extra_c4, last launch). Per workgroup, us after the earliest entry: 0 entry, 1 LLRs
staged in LDS, 2 circular fill done, 3 zero fill done and every store drained.

usage: python tools/diag_dm.py [lib suffix, default diagdm] [symbols]"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{sys.argv[1] if len(sys.argv) > 1 else 'diagdm'}.so"
L = _lib.load()
import bench  # noqa: E402

ctx = _lib.Context(0)
stream = torch.cuda.Stream()
print(bench.extra_c4(ctx, stream, reps=3, from_symbols=len(sys.argv) > 2))
L.ldpc_hip_diag2_read.restype = ctypes.c_int
L.ldpc_hip_diag2_read.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
b = (ctypes.c_uint64 * 8192)()
L.ldpc_hip_diag2_read(b, 8192)
a = np.array(b, dtype=np.int64).reshape(1024, 8)[:, :4]
a = a[a[:, 0] != 0]
t0 = a[:, 0].min()
us = (a - t0) * 0.01
print(f"{len(a)} workgroups; us after the first entry (min / median / max):")
for k, name in enumerate(["entry", "staged", "fill", "drained"]):
    print(f"  {name:8s} {us[:, k].min():6.2f} {np.median(us[:, k]):6.2f} {us[:, k].max():6.2f}")
d = np.diff(us, axis=1)
for k, name in enumerate(["entry->staged", "staged->fill", "fill->drained"]):
    print(f"  {name:14s} {d[:, k].min():6.2f} {np.median(d[:, k]):6.2f} {d[:, k].max():6.2f}")
ctx.close()
