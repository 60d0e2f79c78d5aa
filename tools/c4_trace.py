#!/usr/bin/env python3
"""Diagnostic: runs only bench.py's C4 slot from symbols (default) or from LLRs (argument "llrs"), graph replays, decode launched mixed or per group (argument "nomixed"), for
a rocprofv3 kernel trace of one replayed slot (tools/trace_c4.sh; timeline by tools/trace_timeline.py)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from srsran_projectvtlmo_amd import _lib  # noqa: E402

flags = _lib.LAUNCH_NO_MIXED if "nomixed" in sys.argv[1:] else 0
ctx = _lib.Context(0, launch_flags=flags)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
print(json.dumps(bench.extra_c4(ctx, s, reps=3, from_symbols="llrs" not in sys.argv[1:])))
ctx.close()
