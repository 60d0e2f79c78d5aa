#!/usr/bin/env python3
"""Diagnostic (not product): tests/test_gpu_decoder.py::test_specialised_graph_batch's cases for the given graphs with
a given decoder library (experiment builds), bit-exact vs the oracle.

usage: python tools/check_spec_graphs.py <lib.so> bg:Z[,bg:Z...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = Path(sys.argv[1]).resolve()
import test_gpu_decoder as T  # noqa: E402

ctx = _lib.Context(0)
for item in sys.argv[2].split(","):
    bg, z = (int(x) for x in item.split(":"))
    T.test_specialised_graph_batch(ctx, bg, z)
    print(f"BG{bg} Z={z}: specialised batch bit-exact", flush=True)
ctx.close()
