#!/usr/bin/env python3
"""Diagnostic (not product): does ANY resident grid beside C2 cost what resident work-queue grids do (tools/
dwq_tax_ab.py: +24% with 4 grids = 128 workgroups each owning a CU)? A sleeper grid (tools/ubench/resident_tax.hip)
with the work-queue grid's shape (workgroups, threads, LDS) is launched on its own stream for a few ms, and C2 is timed
beside it with HIP events (10 launches, per-launch time; rounds of 10, median), and per launch.

usage: python tools/resident_tax_ab.py [variant ...]"""
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

VARIANTS = [
    # name, workgroups per sleeper grid, threads, lds bytes, mode, sleeper grids (each on its own stream), stream kind
    ("none", 0, 768, 0, 0, 0, "plain"),
    ("q1_plain_wg128_mode0", 128, 768, 84 * 1024, 0, 1, "plain"),
    ("q1_masked_wg128_mode0", 128, 768, 84 * 1024, 0, 1, "masked"),
    ("q1_masked_wg128_mode2", 128, 768, 84 * 1024, 2, 1, "masked"),
    ("q2_masked_wg64_mode2", 64, 768, 84 * 1024, 2, 2, "masked"),
    ("q3_masked_wg32_mode0", 32, 768, 84 * 1024, 0, 3, "masked"),
    ("q3_masked_wg32_mode2", 32, 768, 84 * 1024, 2, 3, "masked"),
    ("q4_masked_wg32_mode0", 32, 768, 84 * 1024, 0, 4, "masked"),
    ("q4_masked_wg32_mode2", 32, 768, 84 * 1024, 2, 4, "masked"),
    ("q4_masked_wg8_mode0", 8, 768, 84 * 1024, 0, 4, "masked"),
    ("q8_masked_wg16_mode0", 16, 768, 84 * 1024, 0, 8, "masked"),
    ("q4_masked_wg32_t64_lds0_mode0", 32, 64, 0, 0, 4, "masked"),
]


def main():
    import torch

    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    lib = ctypes.CDLL(str(ROOT / "tools" / "ubench" / "libresident_tax.so"))
    lib.launch_sleeper.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    ctx = _lib.Context(0)
    specs, ls, os_ = cc.uniform_batch_specs(128, 1, 384, 8)
    plan = cc.DecodePlan(ctx, specs)
    d_llr = (torch.randint(0, 2, (128, ls), device="cuda", dtype=torch.int8) * 20 - 10).to(torch.int8)
    d_out = torch.zeros(128 * os_, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1024, dtype=torch.int32, device="cuda")
    host = torch.zeros(64, dtype=torch.int32).pin_memory()
    s_batch = torch.cuda.Stream()
    hip = ctypes.CDLL("libamdhip64.so")

    def make_streams(n, kind):
        out = []
        for _ in range(n):
            if kind == "plain":
                out.append(torch.cuda.Stream().cuda_stream)
            else:
                h = ctypes.c_void_p()
                arr = (ctypes.c_uint32 * 8)(*([0xffffffff] * 8))
                rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, arr)
                assert rc == 0, rc
                out.append(h.value)
        return out
    for _ in range(3):
        plan.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, s_batch.cuda_stream)
    torch.cuda.synchronize()
    out = {}
    pick = set(sys.argv[1:])
    for name, nwg, threads, lds, mode, ngrids, kind in VARIANTS:
        if pick and name not in pick and name != "none":
            continue
        streams = make_streams(ngrids, kind)
        rounds, per = [], []
        for _ in range(6):
            for st in streams:
                rc = lib.launch_sleeper(ctypes.c_void_p(st), nwg, threads, lds, 4000.0, mode,
                                        ctypes.c_void_p(host.data_ptr()), ctypes.c_void_p(sink.data_ptr()))
                if rc != 0:
                    out[name] = f"launch_sleeper rc={rc}"
                    break
            if streams:
                time.sleep(0.0005)  # the sleepers are resident before the batch launches arrive
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
            ev[0].record(s_batch)
            for k in range(10):
                plan.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, s_batch.cuda_stream)
                ev[k + 1].record(s_batch)
            torch.cuda.synchronize()
            per.append([round(ev[k].elapsed_time(ev[k + 1]) * 1e3, 1) for k in range(10)])
            rounds.append(ev[0].elapsed_time(ev[10]) / 10 * 1e3)
        torch.cuda.synchronize()
        if name not in out:
            out[name] = {"median_us": round(statistics.median(rounds), 1), "last_round_per_launch": per[-1]}
        if kind == "masked":
            for st in streams:
                hip.hipStreamDestroy(ctypes.c_void_p(st))
        print(json.dumps({name: out[name]}), flush=True)
    base = out["none"]["median_us"]
    print(json.dumps({"resident_tax_pct": {k: round((v["median_us"] / base - 1) * 100, 1) for k, v in out.items()
                                           if isinstance(v, dict)}}))
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
