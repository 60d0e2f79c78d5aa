#!/usr/bin/env python3
"""Diagnostic (not product): bench.py's C3 extra (1024 BG2 Z=208 CBs, 10 it + CRC24B early stop) with a given decoder
library, plus 8-iteration no-CRC batches of the given graphs (kernel time, parity of a sample vs the oracle).

usage: python tools/time_c3.py <lib.so> [bg:Z,bg:Z,...]"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = Path(sys.argv[1]).resolve()
import bench  # noqa: E402
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402

ctx = _lib.Context(0)
stream = torch.cuda.Stream()
r = bench.extra_c3(ctx, stream)
print(Path(sys.argv[1]).name, "C3", json.dumps(r), flush=True)
if len(sys.argv) > 2:
    sys.argv = [sys.argv[0], sys.argv[1], "sweep", sys.argv[2]]
ctx.close()
