#!/usr/bin/env python3
"""Diagnostic (not product): splits the C2 decoder's raw FETCH_SIZE into a per-codeblock and a per-launch part.

Reads tools/g40.sh's PMC passes (gpurun_out/fetch: FETCH_SIZE and WRITE_SIZE at 8, 64, 128, 256 CBs per launch), fits
raw = a * N + b by least squares and writes profiles/r02/fetch_sweep.txt and profiles/fetch_fit.json, which
tools/collect_profiles.py uses: the x2 gfx950 correction (MI355X_MICROARCH.md, calibrated for 16-B/lane streaming
reads) applies to the per-CB part (the LLR loads); the per-launch part is instruction fetch, one copy of the kernel's
code per XCD L2 (8 x the code size), counted as reported.
"""
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
src = Path(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "fetch")
code_bytes = int(sys.argv[2]) if len(sys.argv) > 2 else 50608  # .text size of ldpc_decode_kernel<true,0> (readelf)


def avg(counter, n):
    v = []
    for f in glob.glob(str(src / f"{counter}_{n}" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ldpc_decode_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                v.append(float(r["Counter_Value"]))
    return sum(v) / len(v) * 1024 if v else None


ns = [n for n in (8, 64, 128, 256) if avg("FETCH_SIZE", n) is not None]
fr = {n: avg("FETCH_SIZE", n) for n in ns}
wr = {n: avg("WRITE_SIZE", n) for n in ns}
mx = sum(ns) / len(ns)
my = sum(fr.values()) / len(ns)
a = sum((n - mx) * (fr[n] - my) for n in ns) / sum((n - mx) ** 2 for n in ns)
b = my - a * mx
lines = ["C2 decoder (specialised BG1 Z=384, 8 it): raw rocprofv3 FETCH_SIZE / WRITE_SIZE per dispatch against the",
         "codeblocks per launch (tools/g40.sh, one --pmc pass per counter and size, bench.py --batch N)", "",
         f"{'CBs':>5} {'FETCH raw B':>12} {'fit a*N+b':>12} {'WRITE B':>10}"]
for n in ns:
    lines.append(f"{n:5d} {fr[n]:12.0f} {a * n + b:12.0f} {wr[n]:10.0f}")
lines += ["", f"per CB:     a = {a:.0f} B raw -> x2 = {2 * a:.0f} B (LLRs 25,344 B + descriptor)",
          f"per launch: b = {b:.0f} B raw; 8 XCD L2s x {code_bytes} B of kernel code = {8 * code_bytes} B "
          "(code on paths not taken is never fetched)",
          f"write per CB: {wr[ns[-1]] / ns[-1]:.0f} B (message 1,056 B + result record)"]
(ROOT / "profiles" / "r02" / "fetch_sweep.txt").write_text("\n".join(lines) + "\n")
(ROOT / "profiles" / "fetch_fit.json").write_text(json.dumps(
    {"per_cb_raw_bytes": round(a), "per_launch_raw_bytes": round(b), "kernel_code_bytes": code_bytes,
     "sizes": ns, "source": "tools/g40.sh + tools/fetch_fit.py"}, indent=1) + "\n")
print("\n".join(lines))
