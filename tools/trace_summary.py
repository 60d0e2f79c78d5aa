#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace --output-format csv run: dispatches, p50 and min duration (us) per
(kernel, workgroups). Usage: trace_summary.py <run_kernel_trace.csv> [name-substring ...]"""
import collections
import csv
import statistics
import sys

if __name__ == "__main__":
    keep = sys.argv[2:]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        n = r["Kernel_Name"].split("(")[0][:80]
        if keep and not any(k in n for k in keep):
            continue
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        d[(n, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d}  p50 {statistics.median(v):9.1f}  min {min(v):9.1f}  {n} x{g}")
