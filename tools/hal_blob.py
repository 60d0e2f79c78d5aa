#!/usr/bin/env python3
"""GPU box: writes bench_hal's input (the C4 slot's rate-matched LLRs, bench.hal_slot_blob) to argv[1], so that
tests/cpp/build/bench_hal can run directly under rocprofv3 (bench.py runs it as a child with a temporary file)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import bench  # noqa: E402
from srsran_projectvtlmo_amd import _lib  # noqa: E402

if __name__ == "__main__":
    ctx = _lib.Context(0)
    Path(sys.argv[1]).write_bytes(bench.hal_slot_blob(ctx, 3))
    ctx.close()
