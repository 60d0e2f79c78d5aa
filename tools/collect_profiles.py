#!/usr/bin/env python3
"""Turns a tools/profile.sh run (gpurun_out/prof) into the committed profile files of a round.

  python tools/collect_profiles.py r02 [gpurun_out/prof]

writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --stats summary of bench.py (kernel trace, per kernel name)
  profiles/<round>_pmc.txt            per-counter average over the C2 decoder's dispatches (one --pmc pass per group)
  profiles/pmc_traffic.json           HBM bytes per C2 launch (FETCH_SIZE with MI355X_MICROARCH.md's gfx950 x2 on the
                                      data part, tools/fetch_fit.py, + WRITE_SIZE) and the SQ instruction counts
                                      bench.py's secondary roofline reads, with the digest of the library's sources
                                      (bench.csrc_digest) that bench.py checks before reporting them
"""
import collections
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from bench import csrc_digest  # noqa: E402  (the build identity bench.py checks before reporting traffic)

rnd = sys.argv[1]
src = Path(sys.argv[2] if len(sys.argv) > 2 else ROOT / "gpurun_out" / "prof")
KERNEL = "ldpc_decode_kernel"  # the C2 hot kernel (specialised BG1 Z=384 body)

stats = sorted(glob.glob(str(src / "trace" / "**" / "run_kernel_stats.csv"), recursive=True))
if stats:
    shutil.copy(stats[-1], ROOT / "profiles" / f"{rnd}_kernel_stats.csv")
trace = sorted(glob.glob(str(src / "trace" / "**" / "run_kernel_trace.csv"), recursive=True))
avg_ns = None
if trace:
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace[-1]))
         if r["Kernel_Name"].startswith(f"void ldpc_hip::{KERNEL}") or KERNEL + "<" in r["Kernel_Name"]]
    if d:
        avg_ns = sum(d) / len(d)

agg = collections.defaultdict(list)
for f in sorted(glob.glob(str(src / "pmc*" / "**" / "run_counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if KERNEL + "<" in r["Kernel_Name"] and "mixed" not in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in agg.items()}
with open(ROOT / "profiles" / f"{rnd}_pmc.txt", "w") as fo:
    fo.write(f"# {rnd}: rocprofv3 --pmc, average per dispatch of {KERNEL} (C2: 128 CBs BG1 Z=384, 8 it)\n")
    for k in sorted(avg):
        fo.write(f"{k:32s} n={len(agg[k]):3d} avg={avg[k]:16.1f}\n")
    if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
        fo.write(f"# SQ_WAIT_ANY / SQ_WAVE_CYCLES = {avg['SQ_WAIT_ANY'] / avg['SQ_WAVE_CYCLES']:.3f}\n")
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
        fo.write(f"# SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES = {avg['SQ_ACTIVE_INST_VALU'] / avg['SQ_WAVE_CYCLES']:.3f}\n")

if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    raw = int(avg["FETCH_SIZE"] * 1024)
    wr = int(avg["WRITE_SIZE"] * 1024)
    fit_path = ROOT / "profiles" / "fetch_fit.json"
    fit = json.loads(fit_path.read_text()) if fit_path.exists() else None
    if fit:
        # the x2 correction is calibrated for 16-B/lane streaming reads (the LLR loads, the split-row table copy); the
        # instruction fetch part of the batch-size fit (kernel code once per XCD L2) is counted as reported
        code = min(fit.get("instruction_fetch_raw_bytes", fit["per_launch_raw_bytes"]), raw)
        rd = 2 * (raw - code) + code
        corr = ("FETCH_SIZE = (per-CB data + per-launch tables) x2 (gfx950 16-B/lane streaming reads) + instruction "
                "fetch (8 XCDs x kernel code) as reported (profiles/fetch_fit.json), KiB -> bytes")
    else:
        code, rd = None, 2 * raw
        corr = "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), KiB -> bytes"
    out = {"round": rnd, "kernel": KERNEL + "<true,true> (specialised BG1 Z=384)",
           "workload": "C2: 128 CBs BG1 Z=384, 8 it",
           "fetch_size_kib_raw": round(avg["FETCH_SIZE"], 1), "write_size_kib_raw": round(avg["WRITE_SIZE"], 1),
           "read_bytes_corrected": rd, "instruction_fetch_bytes": code, "read_bytes_all_x2": 2 * raw,
           "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
           "data_bytes_per_launch": rd + wr - (code or 0),
           "rocprof_avg_kernel_ns": avg_ns, "correction": corr, "csrc_sha256": csrc_digest(),
           "fetch_fit": fit}
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
              "SQ_WAIT_ANY"):
        if k in avg:
            out[k.lower() + "_per_launch"] = int(avg[k])
    (ROOT / "profiles" / "pmc_traffic.json").write_text(json.dumps(out, indent=1) + "\n")
print("kernel avg ns:", avg_ns, "counters:", len(avg))
