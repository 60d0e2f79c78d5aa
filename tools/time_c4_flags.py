#!/usr/bin/env python3
"""Diagnostic (not product): bench.py's C4 extras (from LLRs and from symbols) with the default launch flags and with
per-group decode launches (LDPC_HIP_LAUNCH_NO_MIXED), to see which form a slot's decode prefers."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from srsran_projectvtlmo_amd import _lib  # noqa: E402

for name, flags in (("mixed", 0), ("per-group", _lib.LAUNCH_NO_MIXED), ("mixed", 0), ("per-group", _lib.LAUNCH_NO_MIXED)):
    ctx = _lib.Context(0, launch_flags=flags)
    s = torch.cuda.Stream()
    for sym in (False, True):
        r = bench.extra_c4(ctx, s, reps=10, from_symbols=sym)
        print(name, "symbols" if sym else "llrs", r["us_per_slot"], r["tb_crc_ok"], flush=True)
    ctx.close()
