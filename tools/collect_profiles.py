#!/usr/bin/env python3
"""Copy the rocprofv3 summaries of a tools/profile.sh run (gpurun_out/prof) into profiles/ for round TAG:
  profiles/<TAG>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `bench.py` (C2)
  profiles/<TAG>_pmc.txt            per-counter averages over the decoder dispatches
  profiles/pmc_traffic.json         HBM bytes per decoder launch, read by bench.py as roofline.traffic
HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a 16-B/lane streaming read (the decoder's LLR load), so it is doubled;
WRITE_SIZE is taken as is."""
import collections
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = ROOT / (sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/prof")
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)
shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")

agg = collections.defaultdict(list)
for f in sorted(glob.glob(str(src / "pmc*" / "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "ldpc_decode_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in agg.items()}
with open(dst / f"{tag}_pmc.txt", "w") as fh:
    fh.write("# average over ldpc_decode_kernel dispatches of bench.py (C2: 128 CBs BG1 Z=384, 8 it)\n")
    for k in sorted(avg):
        fh.write(f"{k} {avg[k]:.1f} (n={len(agg[k])})\n")
stats = {r["Name"]: r for r in csv.DictReader(open(src / "trace" / "run_kernel_stats.csv"))}
dec = [r for n, r in stats.items() if "ldpc_decode_kernel" in n]
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    rd = avg["FETCH_SIZE"] * 1024 * 2
    wr = avg["WRITE_SIZE"] * 1024
    out = {"round": tag, "kernel": "ldpc_decode_kernel<true>", "workload": "C2: 128 CBs BG1 Z=384, 8 it",
           "fetch_size_kib_raw": round(avg["FETCH_SIZE"], 1), "write_size_kib_raw": round(avg["WRITE_SIZE"], 1),
           "read_bytes_corrected": int(rd), "write_bytes": int(wr), "hbm_bytes_per_launch": int(rd + wr),
           "rocprof_avg_kernel_ns": float(dec[0]["AverageNs"]) if dec else None,
           "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), KiB -> bytes"}
    # instruction counts per launch (wave-instructions summed over the dispatch): bench.py's secondary (VALU-issue)
    # roofline of the LDS-resident decoder
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES"):
        if k in avg:
            out[k.lower() + "_per_launch"] = int(avg[k])
    (dst / "pmc_traffic.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))
