#!/usr/bin/env python3
"""GPU box: bench.py's extra.hal alone (the C4 slot through the HAL plugins: one accelerator TB by TB, then T = 1, 4, 8
concurrent accelerators sharing one HARQ repository, then the PDSCH encoder). Prints its JSON object."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

import bench  # noqa: E402
from srsran_projectvtlmo_amd import _lib  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ctx = _lib.Context(0)
    print(json.dumps(bench.extra_hal(ctx, torch.cuda.current_stream(), reps=reps)), flush=True)
    ctx.close()
