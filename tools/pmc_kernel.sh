#!/bin/bash
# GPU-box diagnostic: one rocprofv3 --pmc pass (counters as arguments) over tools/time_variant.py on LIB (default:
# the product library); prints per-dispatch averages of the counters for ldpc_decode_kernel.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
LIB=${LIB:-srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip.so}
OUT=gpurun_out/pmc_$(echo "$*" | tr ' ' '_' | cut -c1-60)
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT" -o run -- python3 tools/time_variant.py "$LIB" > "$OUT/log.txt" 2>&1
rc=$?
tail -2 "$OUT/log.txt"
[ $rc -ne 0 ] && exit $rc
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ldpc_decode" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k} {sum(v) / len(v):.1f} (n={len(v)})")
PY
