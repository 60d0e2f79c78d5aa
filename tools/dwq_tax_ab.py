#!/usr/bin/env python3
"""Diagnostic (not product): what resident device-work-queue grids cost a concurrent C2 batch launch, split into its
candidate causes: idle polling alone (grids made resident by one item each, then left idle; their
idle period raised so they stay up to their 50 ms lifetime), items running beside (a helper thread keeps submitting
one-iteration one-CB decodes), and the polling knobs (LDPC_HIP_DWQ_SLOT_TICKS, LDPC_HIP_DWQ_POLL_FLAGS). One process
per variant (the knobs are read once per queue). Per variant: C2's HIP-event time per launch over 10 back-to-back
launches, 8 rounds, median.

usage: python tools/dwq_tax_ab.py [variant ...]      (driver: runs the variants in child processes, prints JSON)
       python tools/dwq_tax_ab.py child N MODE"""
import json
import os
import statistics
import subprocess
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GRAPHS = [(2, 36), (2, 208), (1, 120), (2, 96), (1, 52), (2, 12), (1, 256), (2, 384)]

VARIANTS = {
    "none": (0, "idle", {}),
    "g1_idle": (1, "idle", {}),
    "g1_items": (1, "items", {}),
    "g4_idle": (4, "idle", {}),
    "g4_items": (4, "items", {}),
    "g1_idle_longsleep": (1, "idle", {"LDPC_HIP_DWQ_POLL_FLAGS": "1"}),
    "g4_idle_longsleep": (4, "idle", {"LDPC_HIP_DWQ_POLL_FLAGS": "1"}),
    "g4_items_longsleep": (4, "items", {"LDPC_HIP_DWQ_POLL_FLAGS": "1"}),
    "g1_idle_slot400": (1, "idle", {"LDPC_HIP_DWQ_SLOT_TICKS": "400"}),
    "g4_idle_slot400": (4, "idle", {"LDPC_HIP_DWQ_SLOT_TICKS": "400"}),
    "g4_items_slot400": (4, "items", {"LDPC_HIP_DWQ_SLOT_TICKS": "400"}),
}


def child(n, mode):
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
    c2 = _lib.Context(0)
    dec = cc.ldpc_decoder_hip(c2)
    cases = []
    for bg, z in GRAPHS[:n]:
        llr = (rng.integers(0, 2, cc.BG_N_SHORT[bg] * z) * 20 - 10).astype(np.int8)
        cases.append((bg, z, llr))
    calls = [0]

    def one_round():
        for bg, z, llr in cases:
            cfg = cc.configuration()
            cfg.block_conf.tb_common.base_graph = bg
            cfg.block_conf.tb_common.lifting_size = z
            cfg.algorithm_conf.max_iterations = 1
            dec.decode(np.zeros(cc.message_bytes(bg, z), np.uint8), llr, None, cfg)
            calls[0] += 1

    stop = threading.Event()

    def keep_alive():
        while not stop.is_set():
            one_round()
            time.sleep(0.0005)

    for _ in range(3):                      # warm: plan, queues, grids
        plan.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, stream.cuda_stream)
    torch.cuda.synchronize()
    th = None
    if mode == "items" and n:
        th = threading.Thread(target=keep_alive)
        th.start()
        time.sleep(0.2)
    res = []
    for _ in range(8):
        if mode == "idle" and n:
            one_round()                     # (re)launch the grids; they then idle (their 50 ms lifetime bounds it)
            time.sleep(0.002)
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
    c2.close()
    ctx.close()
    print(json.dumps({"grids": n, "mode": mode, "c2_us_per_launch": [round(x, 1) for x in res],
                      "median_us": round(statistics.median(res), 1), "one_cb_calls": calls[0]}))


def main(names):
    out = {}
    for name in names or list(VARIANTS):
        n, mode, env = VARIANTS[name]
        e = dict(os.environ, LDPC_HIP_DWQ_IDLE_US="1000000" if mode == "idle" else "2000", **env)
        r = subprocess.run([sys.executable, __file__, "child", str(n), mode], capture_output=True, text=True,
                           timeout=240, env=e)
        out[name] = (json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else
                     {"error": f"rc={r.returncode} " + r.stderr[-400:]})
        out[name]["env"] = env
        print(json.dumps({name: out[name]}), flush=True)
        if r.returncode != 0:
            break
    base = out.get("none", {}).get("median_us")
    if base:
        print(json.dumps({"dwq_tax_pct": {k: round((v["median_us"] / base - 1) * 100, 1) for k, v in out.items()
                                          if "median_us" in v}}))


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[1] == "child":
        child(int(sys.argv[2]), sys.argv[3])
    else:
        main(sys.argv[1:])
