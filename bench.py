#!/usr/bin/env python3
"""Benchmark of the MI355X LDPC decode path (BASELINE.json metric: LDPC info-bit Gbps @ BG1 Zc=384, 8 iterations).

One step = one pass of the decoder over one batch of codeblocks resident in HBM: 128 CBs of BG1 Z=384
(25,344 int8 LLRs each, all 46 layers active), 8 iterations, no early termination (configs[1], "C2"). Inputs are the
reference benchmark's distribution, LLR = (rgen() & 1) * 20 - 10 (ldpc_decoder_benchmark.cpp:33,144-145),
generated on the device before the timed region.

Multi-GPU (torch.distributed.run): one process per GPU, each decodes its own batch of 128 CBs (independent cells /
slots; weak scaling, no data-path collective). The gloo group is used only for the barriers around the timed region
and the job time: the latest rank's end minus the earliest rank's start on the node clock (>= the max over ranks
of each rank's own elapsed time).

Rank 0 prints ONE JSON line, the headline, LAST (the contract's keys, roofline, cpu_baseline summary; under 8 KB),
preceded, when extras ran, by one '#'-prefixed digest line of them; the full extras go to --extras-out. See
DESIGN.md "Measurement" and section 10 for the roofline accounting and the output format.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

BG, Z, ITERS = 1, 384, 8
K = 22
INFO_BITS_PER_CB = K * Z            # K*Z - F, F = 0
LLR_BYTES_PER_CB = 66 * Z           # N_short * Z int8 LLRs in
MSG_BYTES_PER_CB = INFO_BITS_PER_CB // 8
STATUS_BYTES_PER_CB = 8             # SURVEY.md §8d accounting (the kernel writes a 4-byte result record)
ALGO_BYTES_PER_CB = LLR_BYTES_PER_CB + MSG_BYTES_PER_CB + STATUS_BYTES_PER_CB  # 26,408 B
EDGES_BG1 = 316
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: 8.0 TB/s spec
CLOCK_HZ = 2.4e9                    # MI355X_MICROARCH.md: max clock
VALU_CYCLES_PER_WAVE_INST = 2       # a wave64 VALU instruction issues over 2 cycles on a SIMD-32 (MI355X_MICROARCH.md)
NUM_CUS = 256
METRIC = "LDPC info-bit Gbps @ BG1 Zc=384, 8 iters; codeblocks/s at 1/2/4/8 GPU"


def csrc_digest() -> str:
    """sha256 over the decoder library's sources (csrc/*.hip, *.h, *.cpp, *.inc, Makefile, in name order): the build
    identity that profiles/pmc_traffic.json records (tools/collect_profiles.py) and the bench line checks, so a
    `traffic` figure is only reported for the build it was measured on."""
    import hashlib
    h = hashlib.sha256()
    src = ROOT / "srsran_projectvtlmo_amd" / "csrc"
    for f in sorted(p for p in src.iterdir() if p.suffix in (".hip", ".h", ".cpp", ".inc") or p.name == "Makefile"):
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128, help="codeblocks per GPU per step (configs[1]: 128)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-reps", type=int, default=10000,
                    help="timed single-CB decodes per CPU thread (R >= 200; the default is about 0.9 s per thread on "
                         "an EPYC 9575F, about 16 CPU-seconds in all at 16 threads)")
    ap.add_argument("--extras", choices=["auto", "off"], default="auto",
                    help="also time C3 (1024 BG2 CBs with CRC early stop) and C4 (a PUSCH slot) on one GPU")
    ap.add_argument("--extras-out", default=str(ROOT / "gpurun_out" / "bench_extras.json"),
                    help="file the full extras (C3, C4 variants, z sweep, HAL and software routes) are written to; "
                         "stdout carries only their summary line and the headline line")
    ap.add_argument("--allow-shared-device", action="store_true",
                    help="rehearsal only: let N ranks share fewer GPUs (the line then says so in config.devices)")
    return ap.parse_args(argv)


def _cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.lower().startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cgroup_cpu_quota():
    """CPUs this process may use per the cgroup's CPU bandwidth limit (cpu.max / cfs quota), or None."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(reps: int = 5000):
    """The CPU port of the decoder (oracle/ldpc_cpu_port.c: ldpc_decoder_generic's semantics, bit-exact with the
    oracle, AVX2-organised like the reference's ldpc_decoder_avx2; kind 'port'), timed the way the reference's
    ldpc_decoder_benchmark times its decoder (tests/benchmarks/phy/upper/channel_coding/ldpc/
    ldpc_decoder_benchmark.cpp:87-189, benchmark_utils.h:156-230): one decoder per thread, `reps` timed single-CB
    decodes per thread, median and 99th percentile of the per-CB latency. BASELINE.md section 3: 1 thread and every
    core of this process's affinity mask, on the benchmark's inputs (BG1 Z=384, 8 iterations, LLR = (rand & 1) * 20
    - 10, mt19937-like seed 0) and, single-threaded, on SURVEY 8d's C2 input set (ii) (a codeword + AWGN:
    quantize(2 (1 - 2b) + N(0, 1), 8))."""
    import concurrent.futures as cf

    import numpy as np

    import oracle as O

    O.lib()
    rng = np.random.default_rng(0)
    naff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpu_quota()
    # the cores this process can run on at once: the cgroup CPU quota when there is one, else the job's CPU share as
    # the launcher states it (OMP_NUM_THREADS; 16 per GPU on the GPU boxes, whose affinity mask lists every core of
    # the machine), else the affinity mask
    share = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    ncores = min(naff, quota or share or naff)
    pm1 = (rng.integers(0, 2, LLR_BYTES_PER_CB) * 20 - 10).astype(np.int8)
    msg = rng.integers(0, 2, INFO_BITS_PER_CB).astype(np.uint8)
    cw = O.ldpc_encode(BG, Z, msg)
    awgn = O.quantize_array((1.0 - 2.0 * cw.astype(np.float32)) * 2.0
                            + rng.standard_normal(cw.size).astype(np.float32), 8.0)

    def run(threads, llr, n):
        # the timing loop runs in C threads (oracle/ldpc_cpu_bench.c): no interpreter between the decodes
        lat, wall = O.bench_port(BG, Z, llr, ITERS, threads, n)
        allv = lat.astype(np.float64).ravel() / 1e3
        ncb = threads * n
        return {"threads": threads, "codeblocks": ncb, "wall_s": round(wall, 3),
                "gbit_per_s": round(ncb * INFO_BITS_PER_CB / wall / 1e9, 5),
                "info_mbit_per_s_per_thread": round(INFO_BITS_PER_CB / float(np.median(allv)), 2),
                "p50_us": round(float(np.median(allv)), 1), "p99_us": round(float(np.percentile(allv, 99)), 1)}

    run(1, pm1, 5)                                   # warm-up (library load, page faults)
    one = run(1, pm1, reps)
    one_awgn = run(1, awgn, reps)
    allc = run(ncores, pm1, reps)
    return {"value": allc["gbit_per_s"], "unit": "Gbit/s", "cores": ncores, "kind": "port",
            "sample": f"{allc['codeblocks']} single-CB decodes (BG1 Z=384, 8 it, +-10 LLRs, {reps} per thread) by the "
                      f"AVX2 CPU port on {ncores} threads (every core this process may use: {naff} in the affinity "
                      f"mask, cgroup CPU quota {quota}, OMP_NUM_THREADS {share}) in {allc['wall_s']} s wall; plus "
                      f"{reps} on 1 thread for each input set",
            "cpu_model": _cpu_model(), "affinity_cores": naff, "cgroup_cpu_quota_cores": quota,
            "job_cpu_share": share,
            "single_core": one, "single_core_awgn_codeword": one_awgn, "all_cores": allc,
            "p50_us": one["p50_us"], "p99_us": one["p99_us"],
            "reference_avx2_survey_info_mbit_per_s_per_core": 16.3}


def slot_blob_cbs(blob: bytes):
    """hal_slot_blob's format (u32 nof_tbs; per TB u32 tbs, bg, Z, F, C, Qm, rv, iters; per CB u32 E, E int8 LLRs) as
    per-CB tuples (bg, Z, F, Qm, rv, iters, crc_poly, llr) for oracle.bench_slot; the CB CRC as select_crc
    (pusch_decoder_impl.cpp:35-46): CRC24B with C > 1, else CRC24A above 3824 bits, else CRC16 (oracle CRC ids)."""
    import struct

    import numpy as np
    ntb, = struct.unpack_from("<I", blob, 0)
    off, cbs = 4, []
    for _ in range(ntb):
        tbs, bg, z, f, c, qm, rv, it = struct.unpack_from("<8I", blob, off)
        off += 32
        poly = 1 if c > 1 else (0 if tbs > 3824 else 3)
        for _ in range(c):
            e, = struct.unpack_from("<I", blob, off)
            off += 4
            cbs.append((bg, z, f, qm, rv, it, poly, np.frombuffer(blob, np.int8, e, off).copy()))
            off += e
    return cbs


def cpu_baseline_sw_route(blob: bytes, reps: int = 20, threads=(1, 4, 8, 16)):
    """The software route's CPU leg, the comparison the "auto" decoder type is decided on: the
    same slot's codeblocks on T host threads in pusch_decoder_impl's per-CB task order (pusch_decoder_impl.cpp:309-382,
    pusch_codeblock_decoder.cpp:35-71), each task the oracle's rate dematcher restatement and the AVX2 decoder port
    (oracle/ldpc_cpu_slot.c; kind "port": the reference's AVX2/AVX-512 decoders cannot be built here). Part of the CPU
    baseline: the oracle is the thing timed here, never the product. T is capped at the cores this process may use."""
    import numpy as np

    import oracle as O
    cbs = slot_blob_cbs(blob)
    naff = len(os.sched_getaffinity(0))
    share = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    ncores = min(naff, _cgroup_cpu_quota() or share or naff)
    out = {"kind": "port", "cores": ncores, "cbs": len(cbs), "reps": reps}
    for mode, dm in (("decoder_only", False), ("dematch_decode", True)):
        res = {}
        for t in threads:
            if t > ncores:
                continue
            slot, dec, dmu, ok = O.bench_slot(cbs, t, reps, dm)
            res[f"T{t}"] = {"slot_us_p50": round(float(np.median(slot)), 1),
                            "slot_us_p99": round(float(np.percentile(slot, 99)), 1),
                            "cb_decode_us_p50": round(float(np.median(dec)), 1),
                            "cb_decode_us_p99": round(float(np.percentile(dec, 99)), 1),
                            "cb_dematch_us_p50": round(float(np.median(dmu)), 1) if dm else 0.0,
                            "cbs_crc_ok": ok}
        out[mode] = res
    return out


def _time(fn, stream, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(stream)
    for _ in range(reps):
        fn()
    ev[1].record(stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1e3  # us


def extra_c3(ctx, stream, reps=20):
    """C3: 1024 CBs BG2 Z=208, message 2056 random bits + CRC24B, encoded on the device, soft bits
    quantize(2 (1 - 2b) + N(0, 1), 8) (seed 2), 10 iterations with CRC24B early stop."""
    import numpy as np
    import torch

    from srsran_projectvtlmo_amd import channel_coding as cc
    from srsran_projectvtlmo_amd import segmentation as S
    from srsran_projectvtlmo_amd import synth
    n, bg, z, it = 1024, 2, 208, 10
    rng = np.random.default_rng(2)
    msgs = np.zeros((n, 10 * z), np.uint8)
    msgs[:, :2056] = rng.integers(0, 2, (n, 2056))
    for i in range(n):
        c = S.crc_bits("CRC24B", msgs[i, :2056])
        msgs[i, 2056:] = [(c >> (23 - k)) & 1 for k in range(24)]
    llr = synth.codeword_llrs(ctx, bg, z, msgs, 2.0, 1.0, seed=2)
    specs, ls, os_ = cc.uniform_batch_specs(n, bg, z, it, None, cc.CRC_MODE_EARLY_STOP, cc.CRC24B)
    d_llr = torch.zeros((n, ls), dtype=torch.int8, device="cuda")
    d_llr[:, : llr.shape[1]] = llr
    d_out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    plan = cc.DecodePlan(ctx, specs)
    us = _time(lambda: plan.launch(d_llr.data_ptr(), d_out.data_ptr(), d_res.data_ptr(), stream.cuda_stream), stream,
               reps)
    res = d_res.cpu().numpy().reshape(-1, 4)
    plan.close()
    return {"workload": "C3: BG2 Zc=208, 1024 CBs, 10 it + CRC24B early stop, AWGN codewords (device-encoded)",
            "us_per_batch": round(us, 1), "codeblocks_per_s": round(n / (us * 1e-6), 1),
            "info_gbit_per_s": round(n * 2080 / (us * 1e-6) / 1e9, 4),
            "crc_pass_fraction": round(float(res[:, 0].mean()), 4),
            "mean_iterations": round(float(res[:, 1].mean()), 3)}


LIFTING_SIZES = (2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44, 48,
                 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288,
                 320, 352, 384)
# base-graph edges of the first rows: 4 layers (the shortest codeblock) and all layers (TS 38.212 Tables 5.3.2-2/-3)
EDGES_OF_LAYERS = {(1, 4): 76, (1, 46): 316, (2, 4): 36, (2, 42): 197}


def extra_z_sweep(ctx, stream, n=128, reps=5):
    """Every (BG, lifting size) x {shortest, longest} codeblock at n CBs per launch, 8 iterations, no CRC, LLR =
    (rand & 1) * 20 - 10: the loop of ldpc_decoder_benchmark.cpp:94-140 run as 128-CB batches. Per entry: us per
    batch, info Gbit/s, which kernel ran (specialised / generic) and the cost per edge-lane update (us x GPU CUs in use
    / (n x edges x Z x 8)), relative to BG1 Z=384's."""
    import torch

    from srsran_projectvtlmo_amd import channel_coding as cc
    rows = []
    gen = torch.Generator(device="cuda").manual_seed(94)
    for bg in (1, 2):
        k, nmin, nmax = (22, 24, 66) if bg == 1 else (10, 12, 50)
        for z in LIFTING_SIZES:
            for cbl in (nmin * z, nmax * z):
                specs, ls, os_ = cc.uniform_batch_specs(n, bg, z, ITERS, cbl)
                d_llr = torch.zeros((n, ls), dtype=torch.int8, device="cuda")
                d_llr[:, :cbl] = (torch.randint(0, 2, (n, cbl), device="cuda", dtype=torch.int8, generator=gen) * 20
                                  - 10).to(torch.int8)
                d_out = torch.zeros(n * os_, dtype=torch.uint8, device="cuda")
                plan = cc.DecodePlan(ctx, specs)
                us = _time(lambda: plan.launch(d_llr.data_ptr(), d_out.data_ptr(), 0, stream.cuda_stream), stream,
                           reps)
                plan.close()
                layers = (cbl + 2 * z) // z - k
                edges = EDGES_OF_LAYERS[(bg, layers if layers == 4 else (46 if bg == 1 else 42))]
                rows.append([bg, z, cbl, round(us, 2), round(n * k * z / (us * 1e-6) / 1e9, 3),
                             "S" if cc.specialised(bg, z) == 1 else "G",
                             round(us * 1e6 * min(n, NUM_CUS) / (n * edges * z * ITERS), 2)])
    ref = next(r[6] for r in rows if r[0] == 1 and r[1] == 384 and r[2] == 66 * 384)
    for r in rows:
        r.append(round(r[6] / ref, 3))
    return {"workload": f"every (BG, Z) x {{min, max}} cb_len, {n} CBs, 8 it, no CRC (ldpc_decoder_benchmark loop)",
            "columns": ["bg", "z", "cb_len", "us_per_batch", "info_gbit_per_s", "kernel (S specialised, G generic)",
                        "ps_per_edge_lane_cu", "rel_cost"],
            "unit_note": "ps_per_edge_lane_cu = kernel time x CUs in use / (CBs x edges x Z x iterations); rel_cost "
                         "relative to BG1 Z=384 at the longest cb_len", "rows": rows}


def extra_c4(ctx, stream, reps=20, seed=3, from_symbols=False, amp=2.5, fuse_dematch=True):
    """C4: one 273-PRB n78 slot, 4 layers: UE0 PRB 0-249 256QAM TBS 1,078,248 (128 BG1 CBs, Z=384) and
    23 one-PRB QPSK UEs with TBS 256 (BG2, Z=36, F=88, CRC16); rv 0, new data, soft bits from device-encoded,
    rate-matched codewords with quantize(amp (1 - 2b) + N(0, 1), 8) (seed 3; amp 2.5, where every TB passes; at
    SURVEY 8d's amp of 2.0 the code-rate-0.87 TB of UE0 fails its CRC, reported separately as extra.c4_recipe).
    Timed: rate dematch -> decode (8 it, CRC early stop) -> TB join, all on the device
    (srsran_projectvtlmo_amd.pusch.SlotPipeline).
    from_symbols: the same slot fed with equalised symbols instead (TS 38.211 modulation + complex AWGN, noise
    variance 0.0015 for 256QAM and 0.1 for QPSK), so the timed chain starts with the soft demodulator (§8 f4)."""
    import numpy as np

    from srsran_projectvtlmo_amd import pusch
    from srsran_projectvtlmo_amd import segmentation as S
    from srsran_projectvtlmo_amd import synth
    rng = np.random.default_rng(seed)
    ues = [(1078248, 1, 250 * 156 * 4, 8, 4)] + [(256, 2, 156 * 4, 2, 4)] * 23
    specs, llrs, total = [], [], 0
    for k, (tbs, bg, syms, qm, layers) in enumerate(ues):
        metas = S.segment_rx(tbs, bg, syms, qm, layers)
        m0 = metas[0]
        msgs = S.segment_tx(rng.integers(0, 2, tbs).astype(np.uint8), metas)
        specs.append(pusch.tb_slot_spec(tbs, bg, m0.lifting_size, m0.nof_filler_bits, [m.rm_length for m in metas],
                                        qm, 0, True, 0, 8, True))
        if from_symbols:
            llrs.append(synth.rate_matched_symbols(ctx, bg, m0.lifting_size, msgs, [m.rm_length for m in metas], qm,
                                                   0, m0.nof_filler_bits, 0.0015 if qm == 8 else 0.1, seed=seed + k))
        else:
            llrs.append(synth.rate_matched_llrs(ctx, bg, m0.lifting_size, msgs, [m.rm_length for m in metas], qm, 0,
                                                m0.nof_filler_bits, amp, 1.0, seed=seed + k))
        total += tbs
    pipe = pusch.SlotPipeline(ctx, specs, fuse_dematch=fuse_dematch)
    if from_symbols:
        pipe.upload_symbols_device([a for a, _ in llrs], [b for _, b in llrs])
    else:
        pipe.upload_device(llrs)
    us_eager = _time(lambda: pipe.launch(stream.cuda_stream), stream, reps)
    # the slot recorded once as a HIP graph and replayed: one submission per slot instead of one per kernel
    pipe.capture(stream.cuda_stream)
    us_graph = _time(lambda: pipe.launch_graph(stream.cuda_stream), stream, reps)
    # the headline is one fixed launch form, eager launches back to back (on ROCm 7.0 a graph replay adds a ~8 us gap
    # between replays); the graph-replay time is reported beside it
    us = us_eager
    got, cbres = pipe.results()
    pipe.release_graph()
    return {"workload": "C4: n78 100 MHz 4-layer slot, 24 TBs / 151 CBs mixed BG1/BG2, "
                        + ("soft demodulation + " if from_symbols else "") + "dematch + decode (8 it, ET) "
                        "+ TB join on device" + (f" (cell seed {seed})" if seed != 3 else ""),
            "us_per_slot": round(us, 1), "us_per_slot_eager": round(us_eager, 1),
            "us_per_slot_graph": round(us_graph, 1),
            "launch": "eager launches (back to back); us_per_slot_graph: the same slot replayed as a HIP graph",
            "tb_payload_gbit_per_s": round(total / (us * 1e-6) / 1e9, 4),
            "goodput_gbit_per_s": round(sum(u[0] for u, g in zip(ues, got) if g[1]) / (us * 1e-6) / 1e9, 4),
            "codeblocks": int(cbres.shape[0]), "tb_crc_ok": int(sum(1 for g in got if g[1])), "tbs": len(got),
            "mean_iterations": round(float(cbres[:, 1].mean()), 3), "amplitude": amp,
            "tb_crc": "".join("1" if g[1] else "0" for g in got),
            "cb_crc_ok": int(cbres[:, 0].sum()),
            "iteration_histogram": {int(k): int(v) for k, v in zip(*np.unique(cbres[:, 1], return_counts=True))}}


def extra_sw_route(ctx, stream, reps=20, seed=3, blob=None, cpu_leg=True):
    """The software-factory route, the one the untouched upper PHY builds (upper_phy_factories.cpp:394-445): the C4
    slot's 151 codeblocks as pusch_decoder_impl's per-CB tasks on T worker threads (pusch_decoder_impl.cpp:309-382),
    each thread with its own ldpc_rate_dematcher_hip + ldpc_decoder_hip pair (pusch_decoder_impl.h:48), each task
    pusch_codeblock_decoder::decode's order (rate_dematch into the host soft buffer, then decode with CRC early stop,
    pusch_codeblock_decoder.cpp:35-71). Host buffers in and out, one call per CB. Two pairings: gpu_pair (both on the
    GPU) and decoder_only (soft buffers dematched beforehand: the "auto" pairing, CPU dematcher time not included).
    Run by tests/cpp/build/bench_sw (C++ callers of the C++ adapters). Never `value`."""
    import subprocess
    import tempfile

    exe = ROOT / "tests" / "cpp" / "build" / "bench_sw"
    if not exe.exists():
        return {"error": "tests/cpp/build/bench_sw not built"}
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(blob if blob is not None else hal_slot_blob(ctx, seed))
        path = f.name
    try:
        r = subprocess.run([str(exe), path, str(reps), str(torch_device_index()), "1,4,8,16"], capture_output=True,
                           text=True, timeout=300)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        return {"error": f"bench_sw rc={r.returncode}: {r.stderr[-300:]}"}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["workload"] = ("C4 slot (24 TBs, 151 CBs) through ldpc_rate_dematcher_hip + ldpc_decoder_hip, one call per "
                       "CB from T threads (one decoder pair per thread), host buffers, 8 it + CRC early stop; p50/p99 "
                       "over reps")
    if cpu_leg:
        # the same slot and schedule on the host CPU (the CPU baseline of this route)
        cpu = cpu_baseline_sw_route(blob if blob is not None else hal_slot_blob(ctx, seed), reps)
        out["cpu"] = cpu
        out["gpu_over_cpu_decoder_only"] = {
            t: round(cpu["decoder_only"][t]["slot_us_p50"] / out["decoder_only"][t]["slot_us_p50"], 3)
            for t in cpu["decoder_only"] if t in out.get("decoder_only", {})}
    return out


def extra_hal(ctx, stream, reps=20, seed=3, blob=None):
    """The HAL route, host buffers in and out (PCIe included): the C4 slot's 24 TBs through the PUSCH decoder plugin
    in pusch_decoder_hw_impl's call order with external HARQ, timed per TB and per slot like
    pusch_decoder_hwacc_benchmark.cpp:383-502; the same TBs through the PDSCH encoder plugin in TB and CB mode
    (pdsch_encoder_hwacc_benchmark.cpp). Run by tests/cpp/build/bench_hal (C++ callers of the C++ adapters, so the
    numbers carry no Python overhead), fed with device-generated rate-matched codeword LLRs written to a temp file.
    This rate is never `value`."""
    import subprocess
    import tempfile

    exe = ROOT / "tests" / "cpp" / "build" / "bench_hal"
    if not exe.exists():
        return {"error": "tests/cpp/build/bench_hal not built"}
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(blob if blob is not None else hal_slot_blob(ctx, seed))
        path = f.name
    try:
        r = subprocess.run([str(exe), path, str(reps), str(torch_device_index())], capture_output=True, text=True,
                           timeout=300)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        return {"error": f"bench_hal rc={r.returncode}: {r.stderr[-300:]}"}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["workload"] = ("C4 slot (24 TBs, 151 CBs) through the HAL plugins from host memory: PUSCH decoder "
                       "(reserve -> configure/enqueue x C -> dequeue spin + read outputs -> free, external HARQ, 8 it "
                       "+ ET) and PDSCH encoder (TB mode and CB mode), C++ callers, p50/p99 over reps")
    return out


def hal_slot_blob(ctx, seed=3) -> bytes:
    """The C4 slot's rate-matched codeword LLRs (device-generated, as extra_c4) in bench_hal's input format."""
    import struct

    import numpy as np

    from srsran_projectvtlmo_amd import segmentation as S
    from srsran_projectvtlmo_amd import synth
    rng = np.random.default_rng(seed)
    ues = [(1078248, 1, 250 * 156 * 4, 8, 4)] + [(256, 2, 156 * 4, 2, 4)] * 23
    blob = [struct.pack("<I", len(ues))]
    for k, (tbs, bg, syms, qm, layers) in enumerate(ues):
        metas = S.segment_rx(tbs, bg, syms, qm, layers)
        m0 = metas[0]
        msgs = S.segment_tx(rng.integers(0, 2, tbs).astype(np.uint8), metas)
        llrs = synth.rate_matched_llrs(ctx, bg, m0.lifting_size, msgs, [m.rm_length for m in metas], qm, 0,
                                       m0.nof_filler_bits, 2.5, 1.0, seed=seed + k)
        blob.append(struct.pack("<8I", tbs, bg, m0.lifting_size, m0.nof_filler_bits, len(metas), qm, 0, 8))
        for t in llrs:
            a = t.cpu().numpy().astype(np.int8)
            blob.append(struct.pack("<I", a.size) + a.tobytes())
    return b"".join(blob)


def torch_device_index() -> int:
    import torch
    return torch.cuda.current_device()


HEADLINE_MAX_BYTES = 8192
EXTRAS_PREFIX = "# extras digest: "
HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data", "config", "roofline", "secondary_roofline", "cpu_baseline")


def cpu_baseline_summary(cb):
    """The headline's cpu_baseline object: the contract's keys plus the single-thread latency; the per-leg detail goes
    to the extras file."""
    if not cb:
        return cb
    keep = ("value", "unit", "cores", "kind", "sample", "cpu_model", "p50_us", "p99_us")
    out = {k: cb[k] for k in keep if k in cb}
    if "single_core" in cb:
        out["single_core_gbit_per_s"] = cb["single_core"]["gbit_per_s"]
    if "single_core_awgn_codeword" in cb:
        out["single_core_awgn_p50_us"] = cb["single_core_awgn_codeword"]["p50_us"]
    return out


def label_auto_route(sw):
    """bench_sw's "auto" pairing decides per call between the GPU and a CPU decoder; in this tree the CPU side is the
    oracle's AVX2-organised port (oracle/ldpc_cpu_port.c), not the reference's ldpc_decoder_avx2/avx512. When no call
    went to the GPU the figures are the port's, so the block is renamed to say so."""
    auto = sw.get("auto_decoder_only")
    if not isinstance(auto, dict):
        return sw
    calls = [v for k, v in auto.items() if k.endswith("_calls")]
    gpu_calls = sum(int(c.get("gpu", 0)) for c in calls)
    auto["cpu_decoder"] = "oracle/ldpc_cpu_port.c (test-infrastructure port; a deployment's CPU side is the " \
                          "reference's AVX2/AVX-512 decoder, so LDPC_HIP_AUTO_MIN_WORK must be re-calibrated there)"
    if calls and gpu_calls == 0:
        sw["auto_decoder_only_all_calls_on_cpu_port"] = sw.pop("auto_decoder_only")
    return sw


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def extras_summary(extra):
    """A few-KB digest of the extras for stdout (the full record goes to --extras-out)."""
    s = {}
    for k in ("c3",):
        if k in extra:
            s[k] = _pick(extra[k], ("us_per_batch", "info_gbit_per_s", "crc_pass_fraction", "mean_iterations"))
    for k in ("c4", "c4_recipe", "c4_symbols"):
        if k in extra:
            s[k] = _pick(extra[k], ("us_per_slot", "us_per_slot_graph", "tb_payload_gbit_per_s", "tb_crc_ok", "tbs",
                                    "mean_iterations"))
    if "z_sweep" in extra and "rows" in extra["z_sweep"]:
        rows = extra["z_sweep"]["rows"]
        worst = max(rows, key=lambda r: r[7])
        pick = [r for r in rows if (r[0], r[1]) in ((1, 384), (2, 208), (2, 36))]
        s["z_sweep"] = {"rows": len(rows), "columns": extra["z_sweep"]["columns"], "selected": pick, "worst": worst}
    hal = extra.get("hal")
    if isinstance(hal, dict):
        if "error" in hal:
            s["hal"] = hal
        else:
            h = {"pusch_dec": _pick(hal.get("pusch_dec", {}), ("slot_us_p50", "slot_us_p99", "tb0_us_p50",
                                                                "cbs_crc_ok")),
                 "pusch_dec_phases_us_p50": hal.get("pusch_dec_phases_us_p50"),
                 "pusch_dec_concurrent_slot_us_p50": {t: v.get("slot_us_p50") for t, v in
                                                      hal.get("pusch_dec_concurrent", {}).items()},
                 "pdsch_enc": _pick(hal.get("pdsch_enc", {}), ("tb_mode_slot_us_p50", "cb_mode_slot_us_p50"))}
            s["hal"] = h
    sw = extra.get("sw_route")
    if isinstance(sw, dict):
        if "error" in sw:
            s["sw_route"] = sw
        else:
            o = {}
            for mode in ("gpu_pair", "decoder_only", "auto_decoder_only", "auto_decoder_only_all_calls_on_cpu_port"):
                if mode in sw:
                    o[mode] = {t: [v.get("slot_us_p50"), v.get("cb_decode_us_p50")] for t, v in sw[mode].items()
                               if t[1:].isdigit()}
            o["columns"] = ["slot_us_p50", "cb_decode_us_p50"]
            if "cpu" in sw:
                o["cpu_port_decoder_only"] = {t: [v.get("slot_us_p50"), v.get("cb_decode_us_p50")]
                                              for t, v in sw["cpu"].get("decoder_only", {}).items()}
            if "gpu_over_cpu_decoder_only" in sw:
                o["gpu_over_cpu_decoder_only"] = sw["gpu_over_cpu_decoder_only"]
            s["sw_route"] = o
    if "c5" in extra:
        s["c5"] = extra["c5"]
    return s


def headline_line(*, gbps, world, steps, warmup, elapsed, kernel_ms, n, total_cbs, traffic, prov, secondary,
                  cpu_base, devices=None, devices_distinct=None):
    """The one JSON line the driver parses (the contract's keys; kept under HEADLINE_MAX_BYTES — round 5's 21.5 KB
    line carrying every extra was not parsed)."""
    achieved = ALGO_BYTES_PER_CB * n / (kernel_ms * 1e-3) / 1e9
    cfg = {"workload": "C2: BG1 Zc=384, 128 CBs per GPU, 8 iterations, no early stop, int8 LLR",
           "base_graph": BG, "lifting_size": Z, "iterations": ITERS, "cbs_per_gpu_per_step": n,
           "parallelism": f"cb-batch sharding x{world} (no collective)",
           "job_batch": world * n, "shard_rule": "rank g: codeblocks [g N / G, (g + 1) N / G) (multi_gpu.shard)"}
    if devices is not None:
        cfg["devices"] = devices
        cfg["devices_distinct"] = devices_distinct
    line = {
        "metric": METRIC,
        "value": round(gbps, 4),
        "unit": "Gbit/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic: LLR = (rand & 1) * 20 - 10, resident in HBM (reference benchmark distribution)",
        "config": cfg,
        "codeblocks_per_s": round(total_cbs / elapsed, 1),
        "edge_lane_updates_per_s": round(total_cbs * EDGES_BG1 * Z * ITERS / elapsed, 1),
        "kernel_ms_per_step": round(kernel_ms, 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "algorithmic_bytes_per_launch": ALGO_BYTES_PER_CB * n, "traffic_source": prov},
        "secondary_roofline": secondary,
        "cpu_baseline": cpu_baseline_summary(cpu_base),
    }
    return line


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    # one GPU per rank: local rank -> visible device (modulo the visible count, which also covers a launcher that
    # gives every rank one visible GPU); whether the ranks really drive distinct GPUs is decided below from their
    # physical identities (PCI location / UUID), and a shared GPU is an error unless --allow-shared-device (a
    # multi-rank rehearsal on a 1-GPU box, which the line's config.devices then shows)
    ndev = torch.cuda.device_count()
    local = local % ndev if ndev > 0 else local
    torch.cuda.set_device(local)
    from srsran_projectvtlmo_amd.multi_gpu import check_distinct_devices, device_identity, gather_objects
    devices = gather_objects(dict(device_identity(local), rank=rank)) if world > 1 else None
    distinct = check_distinct_devices(devices, args.allow_shared_device) if devices else None

    from srsran_projectvtlmo_amd import _lib
    from srsran_projectvtlmo_amd import channel_coding as cc

    ctx = _lib.Context(local)
    n = args.batch
    specs, llr_stride, out_stride = cc.uniform_batch_specs(n, BG, Z, ITERS)
    plan = cc.DecodePlan(ctx, specs)
    # the job's batch is world x n codeblocks; rank g decodes the slice [g N / G, (g + 1) N / G) of it (SURVEY 8e's
    # partition rule, multi_gpu.shard), whose LLRs are generated from the slice's start index
    from srsran_projectvtlmo_amd.multi_gpu import shard
    first, last = shard(world * n, rank, world)
    assert last - first == n
    gen = torch.Generator(device="cuda").manual_seed(1234 + first)
    d_llr = (torch.randint(0, 2, (n, llr_stride), device="cuda", dtype=torch.int8, generator=gen) * 20 - 10)
    d_llr = d_llr.to(torch.int8).contiguous()
    d_out = torch.zeros(n * out_stride, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
    # a dedicated (non-null) stream: the kernels and the timing events are on the same HIP stream
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    assert sh != 0

    def step():
        plan.launch(d_llr.data_ptr(), d_out.data_ptr(), d_res.data_ptr(), sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # HIP events on the launch stream around the K back-to-back launches (no marker between launches): the average
    # GPU time per launch, inter-launch gap included (rocprofv3's per-dispatch average is the same within ~1%)
    ev_start = torch.cuda.Event(enable_timing=True)
    ev_end = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the job's wall time on the node's common clock (CLOCK_REALTIME; every rank runs on this node): from the EARLIEST
    # rank's start to the LATEST rank's end, so the skew with which ranks leave the start barrier counts as job time
    w0 = time.time()
    t0 = time.perf_counter()
    ev_start.record(stream)
    for _ in range(args.steps):
        step()
    ev_end.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    w1 = time.time()
    if world > 1:
        dist.barrier()
    kernel_ms = ev_start.elapsed_time(ev_end) / args.steps

    from srsran_projectvtlmo_amd.multi_gpu import job_window, max_over_ranks
    if world > 1:
        elapsed = job_window(w0, w1)             # max(end) - min(start) over ranks
    kernel_ms = max_over_ranks([kernel_ms])[0]

    total_cbs = world * n * args.steps
    gbps = total_cbs * INFO_BITS_PER_CB / elapsed / 1e9
    # traffic (and the PMC instruction counts below) only from a PMC collection of THIS build's sources; a stale file
    # is reported as such, with traffic null
    traffic, pmcd, prov = None, {}, None
    pmc = ROOT / "profiles" / "pmc_traffic.json"
    if pmc.exists():
        try:
            pmcd = json.loads(pmc.read_text())
        except ValueError:
            pmcd = {}
        same = pmcd.get("csrc_sha256") == csrc_digest()
        prov = {"file": "profiles/pmc_traffic.json", "round": pmcd.get("round"), "same_build": same,
                "csrc_sha256": pmcd.get("csrc_sha256"), "rocprof_avg_kernel_ns": pmcd.get("rocprof_avg_kernel_ns")}
        if same:
            traffic = pmcd.get("hbm_bytes_per_launch")
        else:
            pmcd = {}
    # The decoder is LDS-resident: HBM is the metric's roofline but not its bound. The bound that applies is VALU
    # issue on the CUs holding a CB (one CB per CU; the PMC counters in profiles/ are of the same kernel):
    #  * frac: VALU busy time, PMC SQ_ACTIVE_INST_VALU (cycles a wave spends executing VALU instructions, in units of
    #    4 cycles, summed over waves) over those CUs' SIMD cycles in the live kernel time. It weighs each instruction
    #    by its issue cost (most of this kernel's are half-rate packed or 3-operand forms, 4 cycles per wave64);
    #  * issue_frac: PMC SQ_INSTS_VALU against the full-rate issue peak (2 cycles per wave64 instruction), which
    #    counts every instruction as full rate and so reads low for this mix.
    secondary = None
    valu = pmcd.get("sq_insts_valu_per_launch")
    act = pmcd.get("sq_active_inst_valu_per_launch")
    if valu and act:
        cus = min(n, NUM_CUS)
        simd_cycles = cus * 4 * CLOCK_HZ * kernel_ms * 1e-3
        busy = act * 4 / simd_cycles
        v_ach = valu / (kernel_ms * 1e-3)
        v_peak = cus * 4 * CLOCK_HZ / VALU_CYCLES_PER_WAVE_INST
        secondary = {"bound": "valu", "achieved": round(act * 4 / (kernel_ms * 1e-3), 1),
                     "peak": round(cus * 4 * CLOCK_HZ, 1), "unit": "VALU-busy SIMD cycles/s", "frac": round(busy, 4),
                     "issue_frac": round(v_ach / v_peak, 4), "cus": cus,
                     "valu_insts_per_launch": valu, "valu_active_cycles_per_launch": act * 4,
                     "lds_insts_per_launch": pmcd.get("sq_insts_lds_per_launch"),
                     "source": "profiles/pmc_traffic.json (rocprofv3 --pmc SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU) / live "
                               "kernel time"}

    extra, cpu_base = {}, None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        cpu_base = cpu_baseline(args.cpu_reps)
        extra["cpu_baseline_detail"] = cpu_base
    if world == 1 and args.extras == "auto":
        extra.update({"c3": extra_c3(ctx, stream), "c4": extra_c4(ctx, stream),
                      # SURVEY 8d's own C4 recipe, quantize(2.0 (1 - 2b) + N(0, 1), 8): the code-rate-0.87 TB of UE0
                      # fails at this SNR, so the slot runs more iterations and the goodput collapses
                      "c4_recipe": extra_c4(ctx, stream, amp=2.0),
                      "c4_symbols": extra_c4(ctx, stream, from_symbols=True),
                      "z_sweep": extra_z_sweep(ctx, stream)})
        blob = hal_slot_blob(ctx)
        extra["hal"] = extra_hal(ctx, stream, blob=blob)
        extra["sw_route"] = label_auto_route(extra_sw_route(ctx, stream, blob=blob,
                                                            cpu_leg=args.cpu_baseline == "auto"))
    if world > 1 and args.extras == "auto":
        # C5 (configs[4]): one 100 MHz cell per GPU (seeds 3..), every rank decodes its own C4 slot; no collective
        c5 = extra_c4(ctx, stream, seed=3 + rank)
        per = gather_objects([c5["us_per_slot"], c5["tb_crc_ok"]])
        mx = max(p[0] for p in per)
        extra["c5"] = {"workload": f"C5: {world} cells x C4 slot, one cell per GPU (no RCCL)",
                       "max_us_per_slot": round(mx, 1), "us_per_slot_by_rank": [p[0] for p in per],
                       "slots_per_s": round(world / (mx * 1e-6), 1),
                       "tb_crc_ok": int(sum(p[1] for p in per)), "tbs": 24 * world}
    if rank == 0:
        line = headline_line(gbps=gbps, world=world, steps=args.steps, warmup=args.warmup, elapsed=elapsed,
                             kernel_ms=kernel_ms, n=n, total_cbs=total_cbs, traffic=traffic, prov=prov,
                             secondary=secondary, cpu_base=cpu_base, devices=devices, devices_distinct=distinct)
        if extra:
            # the full extras to a file; stdout gets a digest line first and the headline LAST (the driver parses it)
            try:
                out = Path(args.extras_out)
                out.parent.mkdir(parents=True, exist_ok=True)
                out.write_text(json.dumps({"headline": line, "extra": extra}, indent=1))
                where = str(out.relative_to(ROOT)) if out.is_relative_to(ROOT) else str(out)
            except OSError as e:
                where = f"not written ({e})"
            # not a JSON line (the contract's one JSON line is the headline): a '#'-prefixed digest for the log tail
            print(EXTRAS_PREFIX + json.dumps({"bench_extras_summary": extras_summary(extra), "full_record": where}),
                  flush=True)
            line["extras_file"] = where
        print(json.dumps(line), flush=True)
    plan.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
