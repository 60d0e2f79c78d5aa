"""GPU box: 128-CB batch times (8 iterations, no CRC, longest codeblock) of a few graphs under a library variant, and
the oracle check of the smoke test, for a schedule A/B (round 6: lanes per check node of the Z = 36 / 40 one-wave
graphs, LDPC_SPEC_QUAD_P4_MAX_Z). Runs bench._time over cc.DecodePlan launches like bench.extra_z_sweep.

usage: python tools/batch_time_lib.py LIB_SUFFIX|- [reps]   ('-': the product library)"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from srsran_projectvtlmo_amd import _lib  # noqa: E402

if sys.argv[1] != "-":
    _lib.LIB_PATH = ROOT / "srsran_projectvtlmo_amd" / "lib" / f"libsrsran_ldpc_hip_{sys.argv[1]}.so"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20


def main():
    import torch

    import bench
    from srsran_projectvtlmo_amd import channel_coding as cc
    import __graft_entry__ as g
    g.smoke()  # bit-exact vs the oracle on this library (C4 slot with its 23 BG2 Z=36 codeblocks included)
    ctx = _lib.Context(0)
    stream = torch.cuda.Stream()
    gen = torch.Generator(device="cuda").manual_seed(94)
    out = {"lib": str(_lib.LIB_PATH.name)}
    n = 128
    for bg, z in ((2, 36), (1, 36), (2, 40), (1, 40), (2, 32)):
        cbl = (66 if bg == 1 else 50) * z
        specs, ls, os_ = cc.uniform_batch_specs(n, bg, z, 8, cbl)
        d_llr = torch.zeros((n, ls), dtype=torch.int8, device="cuda")
        d_llr[:, :cbl] = (torch.randint(0, 2, (n, cbl), device="cuda", dtype=torch.int8, generator=gen) * 20
                          - 10).to(torch.int8)
        d_out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
        plan = cc.DecodePlan(ctx, specs)
        us = bench._time(lambda: plan.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, stream.cuda_stream), stream, reps)
        plan.close()
        out[f"BG{bg}Z{z}"] = round(us, 2)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
