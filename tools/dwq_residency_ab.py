#!/usr/bin/env python3
"""Diagnostic (not product): what resident device-work-queue grids cost a concurrent batch launch. One process per
configuration (the residency budget LDPC_HIP_DWQ_BUDGET is read once per process): N grids are made resident by
one-codeblock decodes of N distinct graphs (each queue key's grid: 32 workgroups, each owning a CU, staying up to 2 ms
idle), then C2's 128-CB BG1 Z=384 plan is timed (HIP events, 10 launches) while a helper thread keeps those grids busy
enough not to leave. With the default budget (128 workgroups) at most 4 grids are resident; LDPC_HIP_DWQ_BUDGET=256
lets 8 in, which leaves no CU for the batch until the grids leave.

usage: python tools/dwq_residency_ab.py            (driver: runs N = 0, 1, 4, 8 in child processes, prints JSON)
       python tools/dwq_residency_ab.py child N"""
import json
import os
import subprocess
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GRAPHS = [(2, 36), (2, 208), (1, 120), (2, 96), (1, 52), (2, 12), (1, 256), (2, 384)]


def child(n):
    import numpy as np
    import torch
    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    rng = np.random.default_rng(1)
    ctx = _lib.Context(0)
    specs, ls, os_ = cc.uniform_batch_specs(128, 1, 384, 8)
    plan = cc.DecodePlan(ctx, specs)
    d_llr = (torch.randint(0, 2, (128, ls), device="cuda", dtype=torch.int8) * 20 - 10).to(torch.int8)
    d_out = torch.zeros(128 * os_, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    stop = threading.Event()
    calls = [0]

    def keep_alive():
        c2 = _lib.Context(0)
        dec = cc.ldpc_decoder_hip(c2)
        cases = []
        for bg, z in GRAPHS[:n]:
            llr = (rng.integers(0, 2, cc.BG_N_SHORT[bg] * z) * 20 - 10).astype(np.int8)
            cases.append((bg, z, llr))
        while not stop.is_set():
            for bg, z, llr in cases:
                cfg = cc.configuration()
                cfg.block_conf.tb_common.base_graph = bg
                cfg.block_conf.tb_common.lifting_size = z
                cfg.algorithm_conf.max_iterations = 1
                dec.decode(np.zeros(cc.message_bytes(bg, z), np.uint8), llr, None, cfg)
                calls[0] += 1
            time.sleep(0.0005)  # well inside the grids' 2 ms idle period
        c2.close()

    th = threading.Thread(target=keep_alive) if n else None
    if th:
        th.start()
        time.sleep(0.2)
    res = []
    for _ in range(5):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(10):
            plan.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, stream.cuda_stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        res.append(ev[0].elapsed_time(ev[1]) / 10 * 1e3)
    stop.set()
    if th:
        th.join(30)
    plan.close()
    ctx.close()
    print(json.dumps({"grids_requested": n, "c2_us_per_launch": [round(x, 1) for x in res],
                      "one_cb_calls_beside": calls[0], "budget": os.environ.get("LDPC_HIP_DWQ_BUDGET", "128")}))


def main():
    out = []
    for n, env in ((0, {}), (1, {}), (4, {}), (8, {}), (8, {"LDPC_HIP_DWQ_BUDGET": "256"})):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, __file__, "child", str(n)], capture_output=True, text=True, timeout=300,
                           env=e)
        out.append(json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else
                   {"grids_requested": n, "error": r.stderr[-400:]})
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"dwq_residency_ab": out}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(int(sys.argv[2]))
    else:
        main()
