#!/usr/bin/env python3
"""Diagnostic (not product): is the work-queue "tax" (tools/dwq_tax_ab.py: C2 +24% with 4 grids = 128 CUs resident,
+3% with 1 grid) a property of a full chip rather than of the grids? C2 (128 CBs of BG1 Z=384, 8 it) timed with HIP
events, 10 launches x 8 rounds, median, as:
  alone          one 128-CB launch on a plain stream (128 of 256 CUs busy)
  b256           one 256-CB launch (every CU holds one CB), time per launch reported per 128 CBs too
  two_streams    two 128-CB launches at once on two streams (every CU busy, two kernels)
  mask_<name>    one 128-CB launch on a CU-masked stream (hipExtStreamCreateWithCUMask; 8 x 32-bit words), with
                 masks that select 128 CUs in different patterns (mask bit order is the runtime's)
usage: python tools/cu_placement_ab.py"""
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def masks():
    def from_bits(bits):
        w = [0] * 8
        for b in bits:
            w[b // 32] |= 1 << (b % 32)
        return w
    return {
        "low128": from_bits(range(128)),
        "high128": from_bits(range(128, 256)),
        "even": from_bits(range(0, 256, 2)),
        "odd": from_bits(range(1, 256, 2)),
        "pairs_even": from_bits([b for b in range(256) if (b // 2) % 2 == 0]),
        "quads_even": from_bits([b for b in range(256) if (b // 4) % 2 == 0]),
        "oct_even": from_bits([b for b in range(256) if (b // 8) % 2 == 0]),
        "b16_even": from_bits([b for b in range(256) if (b // 16) % 2 == 0]),
        "word_even": from_bits([b for b in range(256) if (b // 32) % 2 == 0]),
        "all": [0xffffffff] * 8,
    }


def main():
    import torch

    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc
    hip = ctypes.CDLL("libamdhip64.so")
    ctx = _lib.Context(0)
    specs, ls, os_ = cc.uniform_batch_specs(256, 1, 384, 8)
    plan256 = cc.DecodePlan(ctx, specs)
    plan128 = cc.DecodePlan(ctx, specs[:128])
    d_llr = (torch.randint(0, 2, (256, ls), device="cuda", dtype=torch.int8) * 20 - 10).to(torch.int8)
    d_out = torch.zeros(256 * os_, dtype=torch.uint8, device="cuda")
    d_out2 = torch.zeros(256 * os_, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(launch, streams, rounds=8, reps=10):
        res = []
        for _ in range(rounds + 1):
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(streams[0])
            for s in streams[1:]:
                s.wait_event(ev[0])
            for _ in range(reps):
                launch()
            for s in streams[1:]:
                e = torch.cuda.Event()
                e.record(s)
                streams[0].wait_event(e)
            ev[1].record(streams[0])
            torch.cuda.synchronize()
            res.append(ev[0].elapsed_time(ev[1]) / reps * 1e3)
        return round(statistics.median(res[1:]), 1)

    out = {}
    out["alone"] = timed(lambda: plan128.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, s1.cuda_stream), [s1])
    out["b256"] = timed(lambda: plan256.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, s1.cuda_stream), [s1])

    def two():
        plan128.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, s1.cuda_stream)
        plan128.launch(d_llr.data_ptr(), d_out2.data_ptr(), 0, s2.cuda_stream)
    out["two_streams"] = timed(two, [s1, s2])
    print(json.dumps(out), flush=True)
    for name, m in masks().items():
        h = ctypes.c_void_p()
        arr = (ctypes.c_uint32 * 8)(*m)
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, arr)
        if rc != 0:
            out["mask_" + name] = f"hipExtStreamCreateWithCUMask rc={rc}"
            continue
        st = torch.cuda.ExternalStream(h.value)
        out["mask_" + name] = timed(lambda: plan128.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, h.value), [st])
        torch.cuda.synchronize()
        hip.hipStreamDestroy(h)
        print(json.dumps({name: out["mask_" + name]}), flush=True)
    plan128.close()
    plan256.close()
    ctx.close()
    print(json.dumps({"cu_placement_ab_us_per_launch": out}))


if __name__ == "__main__":
    main()
