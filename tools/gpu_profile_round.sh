#!/bin/bash
# GPU box: the round's committed evidence -- tools/profile.sh (kernel trace + stats and the PMC passes of the C2
# bench), then the default bench line (CPU baseline and extras included). Logs under gpurun_out/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/profile.sh > gpurun_out/profile.txt 2>&1
rc=$?; cat gpurun_out/profile.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_full.log
exit $rc
