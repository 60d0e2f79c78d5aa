#!/usr/bin/env python3
"""Per-variant average of the decode kernel's PMC counters (tools/pmc_variants.sh output)."""
import collections
import csv
import glob
import sys

for d in sorted(glob.glob("gpurun_out/pmcv/*")):
    f = glob.glob(d + "/**/run_counter_collection.csv", recursive=True)
    if not f:
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "decode_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d.split("/")[-1], " ".join(f"{k}={sum(v) / len(v):.4g}" for k, v in sorted(agg.items())))
