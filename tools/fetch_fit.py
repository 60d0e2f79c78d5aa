#!/usr/bin/env python3
"""Diagnostic (not product): splits the C2 decoder's raw FETCH_SIZE into a per-codeblock and a per-launch part, and
the per-launch part into instruction fetch and table reads.

Reads tools/fetch_sweep.sh's PMC passes (gpurun_out/fetch/<lib>/<COUNTER>_<N>: FETCH_SIZE and WRITE_SIZE at 8, 64,
128, 256 CBs per launch; <lib> = "cur", the product library, and "notab", the variant without the split-row address
table), fits raw = a * N + b per library by least squares and writes profiles/r04/fetch_sweep.txt and
profiles/fetch_fit.json, which tools/collect_profiles.py uses:
  * a (per CB): the LLR loads, 16-B/lane streaming reads, so x2 (MI355X_MICROARCH.md's gfx950 correction);
  * b (per launch) = instruction fetch (the code each XCD's L2 fetches once, counted as reported), plus tables every
    XCD reads once (the split-row address table, 16-B loads, so x2). b(notab), the variant without the table, is its
    instruction fetch alone; b(cur) - b(notab) is the split table's share.

usage: python tools/fetch_fit.py [src] --code cur=<bytes> notab=<bytes>   (.text size of ldpc_decode_kernel<true,0>
       of each library: llvm-readelf -s on its gfx950 code object)"""
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
args = sys.argv[1:]
code = {}
if "--code" in args:
    i = args.index("--code")
    code = {k: int(v) for k, v in (a.split("=") for a in args[i + 1:])}
    args = args[:i]
src = Path(args[0] if args else ROOT / "gpurun_out" / "fetch")
SPLIT_TABLE_BYTES = 61440   # BG1 Z=384's split-row address table (20 words x 768 lanes x 4 B), SPLIT_TAB_STRIDE
NS = (8, 64, 128, 256)


def avg(lib, counter, n):
    v = []
    for f in glob.glob(str(src / lib / f"{counter}_{n}" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ldpc_decode_kernel<" in r["Kernel_Name"] and "mixed" not in r["Kernel_Name"] and \
                    r["Counter_Name"] == counter:
                v.append(float(r["Counter_Value"]))
    return sum(v) / len(v) * 1024 if v else None


def fit(lib, counter):
    pts = {n: avg(lib, counter, n) for n in NS}
    pts = {n: y for n, y in pts.items() if y is not None}
    if len(pts) < 2:
        return None
    mx = sum(pts) / len(pts)
    my = sum(pts.values()) / len(pts)
    a = sum((n - mx) * (y - my) for n, y in pts.items()) / sum((n - mx) ** 2 for n in pts)
    return a, my - a * mx, pts


libs = [d.name for d in sorted(src.iterdir()) if d.is_dir()]
res = {lib: fit(lib, "FETCH_SIZE") for lib in libs}
res = {k: v for k, v in res.items() if v}
wr = fit("cur", "WRITE_SIZE")
lines = ["C2 decoder (specialised BG1 Z=384, 8 it): raw rocprofv3 FETCH_SIZE / WRITE_SIZE per dispatch against the",
         "codeblocks per launch (tools/fetch_sweep.sh: one --pmc pass per counter, size and library, 12 launches each)",
         ""]
for lib, (a, b, pts) in res.items():
    lines.append(f"[{lib}]  {'CBs':>5} {'FETCH raw B':>12} {'fit a*N+b':>12}" + (f" {'WRITE B':>10}" if lib == "cur" else ""))
    for n, y in pts.items():
        w = f" {wr[2][n]:10.0f}" if lib == "cur" and wr and n in wr[2] else ""
        lines.append(f"        {n:5d} {y:12.0f} {a * n + b:12.0f}{w}")
    lines.append(f"        per CB a = {a:.0f} B raw -> x2 = {2 * a:.0f} B (LLRs 25,344 B + descriptor); per launch b = {b:.0f} B raw")
    if lib in code:
        lines.append(f"        8 XCD L2s x {code[lib]} B of kernel code = {8 * code[lib]} B")
    lines.append("")
out = {"source": "tools/fetch_sweep.sh + tools/fetch_fit.py", "sizes": list(NS), "libraries": {}}
for lib, (a, b, _) in res.items():
    e = {"per_cb_raw_bytes": round(a), "per_launch_raw_bytes": round(b)}
    if lib in code:
        e["kernel_code_bytes"] = code[lib]
        e["instruction_fetch_raw_bytes"] = min(8 * code[lib], round(b))
        e["per_launch_table_raw_bytes"] = round(b) - e["instruction_fetch_raw_bytes"]
    out["libraries"][lib] = e
if "cur" in res and "notab" in res:
    # the no-table variant's per-launch part is its instruction fetch alone (below 8 x its code size: code on paths a
    # C2 launch never takes is never fetched); the product's code differs from it by 2%, so b(notab) stands for the
    # product's instruction fetch too, and the rest of b(cur) is the split-row table
    d = res["cur"][1] - res["notab"][1]
    cur = out["libraries"]["cur"]
    cur["instruction_fetch_raw_bytes"] = round(res["notab"][1])
    cur["per_launch_table_raw_bytes"] = round(d)
    out["libraries"]["notab"]["instruction_fetch_raw_bytes"] = round(res["notab"][1])
    out["libraries"]["notab"]["per_launch_table_raw_bytes"] = 0
    out["split_table_raw_bytes_per_launch"] = round(d)
    lines.append(f"instruction fetch per launch: b(notab) = {res['notab'][1]:.0f} B (as reported; "
                 f"{res['notab'][1] / (8 * code['notab']):.2f} of 8 x its code)" if "notab" in code else
                 f"instruction fetch per launch: b(notab) = {res['notab'][1]:.0f} B")
    lines.append(f"split-row address table: b(cur) - b(notab) = {d:.0f} B raw -> x2 = {2 * d:.0f} B "
                 f"(8 XCDs x {SPLIT_TABLE_BYTES} B = {8 * SPLIT_TABLE_BYTES} B: each XCD's L2 reads it once, "
                 f"+ {(2 * d - 8 * SPLIT_TABLE_BYTES) / 8:.0f} B per XCD)")
if wr:
    lines.append(f"write per CB: {wr[0]:.0f} B (message 1,056 B + result record), per launch {wr[1]:.0f} B")
cur = out["libraries"].get("cur", {})
out.update({k: cur[k] for k in ("per_cb_raw_bytes", "per_launch_raw_bytes", "kernel_code_bytes",
                                "instruction_fetch_raw_bytes") if k in cur})
(ROOT / "profiles" / "r04").mkdir(parents=True, exist_ok=True)
(ROOT / "profiles" / "r04" / "fetch_sweep.txt").write_text("\n".join(lines) + "\n")
(ROOT / "profiles" / "fetch_fit.json").write_text(json.dumps(out, indent=1) + "\n")
print("\n".join(lines))
