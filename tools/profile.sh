#!/bin/bash
# GPU-box profiling: kernel trace + stats of bench.py, then PMC passes (one counter group per pass, no tracing
# domains beside --kernel-trace, as gpurun requires). Output under gpurun_out/prof/.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
STEPS=${STEPS:-10}
B="bench.py --steps $STEPS --warmup 2 --cpu-baseline off --extras off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 $B > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($grp) rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done < "${PMC_FILE:-tools/pmc_groups.txt}"
exit 0
