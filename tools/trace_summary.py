#!/usr/bin/env python3
"""Diagnostic: per-kernel count / average / total duration (us) of a rocprofv3 kernel trace (default gpurun_out/px)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/px"
f = sorted(glob.glob(f"{root}/**/run_kernel_trace.csv", recursive=True))[-1]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ldpc_hip::", "")
    if "at::" in name or "anonymous" in name:
        continue
    grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
    agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{name[:60]:60s} grid {grid:>8s}  n={len(v):3d}  avg {sum(v) / len(v):8.2f} us  total {sum(v):9.1f} us")
