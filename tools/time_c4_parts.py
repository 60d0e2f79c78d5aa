#!/usr/bin/env python3
"""Diagnostic (not product): the C4 slot (from LLRs, amplitude 2.5) split into its parts -- the whole slot, UE0's
128-CB TB alone, the 23 one-CB TBs alone -- each as a replayed HIP graph, to find the decode's critical path.

usage: python tools/time_c4_parts.py [lib.so] [reps]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1].endswith(".so"):
    _lib.LIB_PATH = Path(sys.argv[1]).resolve()
import bench  # noqa: E402
from srsran_projectvtlmo_amd import pusch, segmentation as S, synth  # noqa: E402

reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = _lib.Context(0)
stream = torch.cuda.Stream()
rng = np.random.default_rng(3)
ues = [(1078248, 1, 250 * 156 * 4, 8, 4)] + [(256, 2, 156 * 4, 2, 4)] * 23
specs, llrs = [], []
for k, (tbs, bg, syms, qm, layers) in enumerate(ues):
    metas = S.segment_rx(tbs, bg, syms, qm, layers)
    m0 = metas[0]
    msgs = S.segment_tx(rng.integers(0, 2, tbs).astype(np.uint8), metas)
    specs.append(pusch.tb_slot_spec(tbs, bg, m0.lifting_size, m0.nof_filler_bits, [m.rm_length for m in metas], qm, 0,
                                    True, 0, 8, True))
    llrs.append(synth.rate_matched_llrs(ctx, bg, m0.lifting_size, msgs, [m.rm_length for m in metas], qm, 0,
                                        m0.nof_filler_bits, 2.5, 1.0, seed=3 + k))
for name, idx in (("slot", list(range(24))), ("UE0 (128 BG1 CBs)", [0]), ("23 one-CB TBs", list(range(1, 24))),
                  ("one one-CB TB", [1])):
    pipe = pusch.SlotPipeline(ctx, [specs[i] for i in idx])
    pipe.upload_device([llrs[i] for i in idx])
    eager = bench._time(lambda: pipe.launch(stream.cuda_stream), stream, reps)
    pipe.capture(stream.cuda_stream)
    us = bench._time(lambda: pipe.launch_graph(stream.cuda_stream), stream, reps)
    got, cbres = pipe.results()
    pipe.release_graph()
    print(f"{name}: graph {us:.1f} us, eager {eager:.1f} us, TB CRC ok {sum(1 for g in got if g[1])}/{len(got)}, "
          f"max it {int(cbres[:, 1].max())}", flush=True)
ctx.close()
