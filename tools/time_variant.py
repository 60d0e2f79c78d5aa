#!/usr/bin/env python3
"""Diagnostic (not product): kernel time of a decoder library variant on the C2 batch.

usage: python tools/time_variant.py <lib.so> [bg] [Z] [iters] [n]
       python tools/time_variant.py <lib.so> sweep bg:Z,bg:Z,...   (several graphs, 8 it, 128 CBs)"""
import sys
from pathlib import Path

import torch  # noqa: F401  (one HIP runtime: torch first)

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

_lib.LIB_PATH = Path(sys.argv[1]).resolve()
from srsran_projectvtlmo_amd import channel_coding as cc  # noqa: E402
import oracle as O  # noqa: E402  (bit-exactness of the variant on the first CBs: test infrastructure, checker only)


def one(ctx, bg, Z, iters, n):
    specs, ls, os_ = cc.uniform_batch_specs(n, bg, Z, iters)
    plan = cc.DecodePlan(ctx, specs)
    g = torch.Generator(device="cuda").manual_seed(1)
    llr = (torch.randint(0, 2, (n, ls), device="cuda", dtype=torch.int8, generator=g) * 20 - 10).to(torch.int8)
    out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for rep in range(12):
        ev[0].record(s)
        plan.launch(llr.data_ptr(), out.data_ptr(), 0, s.cuda_stream)
        ev[1].record(s)
        torch.cuda.synchronize()
        if rep >= 2:
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    plan.close()
    ts.sort()
    h_llr = llr.cpu().numpy()
    h_out = out.cpu().numpy()
    bad = 0
    for i in range(min(n, 3)):
        ref, _ = O.ldpc_decode(bg, Z, h_llr[i, :cc.BG_N_SHORT[bg] * Z], iters)
        bad += int(not (h_out[i * os_:i * os_ + ref.size] == ref).all())
    print(f"{Path(sys.argv[1]).name}: BG{bg} Z={Z} {iters} it {n} CBs: median {ts[len(ts) // 2]:.1f} us min "
          f"{ts[0]:.1f} us parity {'OK' if bad == 0 else f'FAIL ({bad} CBs differ)'}", flush=True)


ctx = _lib.Context(0)
if len(sys.argv) > 2 and sys.argv[2] == "sweep":
    for item in sys.argv[3].split(","):
        b_, z_ = item.split(":")
        one(ctx, int(b_), int(z_), 8, 128)
else:
    one(ctx, int(sys.argv[2]) if len(sys.argv) > 2 else 1, int(sys.argv[3]) if len(sys.argv) > 3 else 384,
        int(sys.argv[4]) if len(sys.argv) > 4 else 8, int(sys.argv[5]) if len(sys.argv) > 5 else 128)
ctx.close()
