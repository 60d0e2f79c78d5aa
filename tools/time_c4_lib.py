#!/usr/bin/env python3
"""Diagnostic (not product): bench.py's C4 slot (from LLRs and from symbols, amplitude 2.5; the dematcher fused into
the decode kernels and as its own kernel) on a given library variant.

usage: python tools/time_c4_lib.py <lib.so> [reps]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = Path(sys.argv[1]).resolve()
import bench  # noqa: E402

reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = _lib.Context(0)
s = torch.cuda.Stream()
fused = [True, False] if hasattr(_lib, "LAUNCH_SEPARATE_DEMATCH") else [True]
for sym in (False, True):
    for fu in fused:
        r = bench.extra_c4(ctx, s, reps=reps, from_symbols=sym, fuse_dematch=fu)
        print(f"{_lib.LIB_PATH.name}: C4 {'symbols' if sym else 'llrs'}{'' if fu else ' (separate dematch)'} "
              f"{r['us_per_slot']} us/slot (graph {r.get('us_per_slot_graph')}, eager {r.get('us_per_slot_eager')}), "
              f"TB CRC ok {r['tb_crc_ok']}/{r['tbs']}, mean it {r['mean_iterations']}", flush=True)
ctx.close()
