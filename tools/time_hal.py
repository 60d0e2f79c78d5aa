#!/usr/bin/env python3
"""Diagnostic (not product): bench.py's HAL-route figures alone (extra_hal: the C4 slot through the PUSCH decoder
plugin, T = 1 / 4 / 8 concurrent instances, and the PDSCH encoder plugin).

usage: python tools/time_hal.py [reps]"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from srsran_projectvtlmo_amd import _lib  # noqa: E402

ctx = _lib.Context(0)
print(json.dumps(bench.extra_hal(ctx, torch.cuda.Stream(), reps=int(sys.argv[1]) if len(sys.argv) > 1 else 20)))
ctx.close()
