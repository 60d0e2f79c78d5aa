#!/usr/bin/env python3
"""Diagnostic (not product): cost per iteration of BG1 Z=384 CBs with the minimum of 4 layers (one non-zero LLR), i.e.
of the four split steps (rows 0-3) alone, for several library variants; slope between 2 and 10 iterations.

usage: python tools/time_split.py lib.so   (one library per process)"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402


def run(path):
    _lib.LIB_PATH = Path(path).resolve()
    from srsran_projectvtlmo_amd import channel_coding as cc
    ctx = _lib.Context(0)
    out = {}
    for layers_nz in (1, 9728):
        t = {}
        for it in (2, 10):
            n = 128
            specs, ls, os_ = cc.uniform_batch_specs(n, 1, 384, it)
            plan = cc.DecodePlan(ctx, specs)
            g = torch.Generator(device="cuda").manual_seed(1)
            llr = torch.zeros((n, ls), device="cuda", dtype=torch.int8)
            llr[:, :layers_nz] = torch.randint(0, 2, (n, layers_nz), device="cuda", dtype=torch.int8,
                                               generator=g) * 20 - 10
            o = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
            s = torch.cuda.Stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for rep in range(12):
                e0.record(s)
                plan.launch(llr.data_ptr(), o.data_ptr(), 0, s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                if rep >= 2:
                    ts.append(e0.elapsed_time(e1) * 1e3)
            plan.close()
            ts.sort()
            t[it] = ts[len(ts) // 2]
        out[layers_nz] = (t[10] - t[2]) / 8
    ctx.close()
    print(f"{Path(path).name}: per iteration 4 layers {out[1]:.2f} us ({out[1] / 4 * 1e3:.0f} ns per split step), "
          f"6 layers {out[9728]:.2f} us", flush=True)


run(sys.argv[1])
