#!/usr/bin/env python3
"""Summarise rocprofv3 PMC CSVs under a directory: per counter, average over dispatches of the decoder kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
pat = sys.argv[2] if len(sys.argv) > 2 else "decode"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:32s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
