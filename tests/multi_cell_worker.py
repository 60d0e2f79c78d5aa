"""One rank of tests/test_gpu_multi_cell.py (launched by torch.distributed.run): C5's one-cell-per-GPU rule
(multi_gpu.cell_to_device) -- rank r decodes cell r's full C4 slot (seed 3 + r) on its own context and checks every
CB and TB against the oracle flow (tests/tb_chain.SwFlow). With fewer GPUs than ranks the ranks share the visible
ones. The gloo group carries only the result count; the data path has no collective."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)   # before any GPU call
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd.multi_gpu import cell_to_device
    from tests.tb_chain import SwFlow
    from tests.test_gpu_c4_full import _c4_tbs, _pipeline
    dev = cell_to_device(rank, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    ctx = _lib.Context(dev)
    rng, tbs = _c4_tbs(3 + rank)
    llrs = [tb.llrs(rng, 0, 2.0, 0.7) for tb in tbs]
    flows = [SwFlow(tb, nof_iters=8, early_stop=True) for tb in tbs]
    expect = [f.transmission(l, 0, True) for f, l in zip(flows, llrs)]
    pipe = _pipeline(ctx, tbs, 8)
    pipe.upload(llrs)
    pipe.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got, cbres = pipe.results()
    bad, i, tb_ok = 0, 0, 0
    for tb, f, (ok, _), (tb_bytes, g_ok, _w) in zip(tbs, flows, expect, got):
        for r in range(tb.C):
            bad += int(bool(cbres[i + r, 0]) != f.crc_ok[r] or int(cbres[i + r, 1]) != f.iters_used[r])
        i += tb.C
        bad += int(g_ok != ok)
        if ok:
            tb_ok += 1
            bad += int(not np.array_equal(np.unpackbits(tb_bytes)[: tb.tbs], tb.data))
    t = torch.tensor([bad, tb_ok], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"ranks": world, "devices": torch.cuda.device_count(), "mismatches": int(t[0]),
                          "tb_crc_ok": int(t[1]), "tbs": 24 * world}), flush=True)
    ctx.close()
    dist.destroy_process_group()
    sys.exit(0 if int(t[0]) == 0 else 1)


if __name__ == "__main__":
    main()
