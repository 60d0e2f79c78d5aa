#!/usr/bin/env python3
"""Diagnostic: timeline (start offset, duration, gap to the previous end) of the last N kernel dispatches of a
rocprofv3 kernel trace (default gpurun_out/px), to see launch gaps inside a replayed slot graph."""
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/px"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
f = sorted(glob.glob(f"{root}/**/run_kernel_trace.csv", recursive=True))[-1]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ldpc_hip::", "")[:48]
    gap = "" if prev_end is None else f"{(s - prev_end) / 1000:8.2f}"
    print(f"{(s - t0) / 1000:9.2f} us  dur {(e - s) / 1000:8.2f}  gap {gap:>8s}  {name}")
    prev_end = e if prev_end is None else max(prev_end, e)
