#!/bin/bash
# GPU box (round 4): the committed perf evidence from ONE build, in order:
#   1. tools/fetch_sweep.sh: FETCH_SIZE / WRITE_SIZE of the C2 decoder at 8-256 CBs per launch, product library and
#      the variant without the split-row address table; tools/fetch_fit.py refits profiles/fetch_fit.json;
#   2. tools/profile.sh: kernel trace + stats of bench.py and the PMC passes (tools/pmc_groups.txt);
#      tools/collect_profiles.py writes profiles/r04_kernel_stats.csv, r04_pmc.txt and pmc_traffic.json (with the
#      sources' digest);
#   3. the default bench line, which reads that pmc_traffic.json (same digest: traffic and the VALU figures reported).
# The profiles/ files written here come back under gpurun_out/profiles/. Usage: gpu_r04_evidence.sh CODE_CUR CODE_NOTAB
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/fetch_sweep.sh notab > gpurun_out/fetch_sweep.log 2>&1
rc=$?; cat gpurun_out/fetch_sweep.log; [ $rc -ne 0 ] && exit $rc
python3 tools/fetch_fit.py gpurun_out/fetch --code cur=$1 notab=$2 || exit 1
bash tools/profile.sh > gpurun_out/profile.txt 2>&1
rc=$?; cat gpurun_out/profile.txt; [ $rc -ne 0 ] && exit $rc
python3 tools/collect_profiles.py r04 gpurun_out/prof || exit 1
mkdir -p gpurun_out/profiles/r04
cp profiles/fetch_fit.json profiles/pmc_traffic.json profiles/r04_kernel_stats.csv profiles/r04_pmc.txt gpurun_out/profiles/
cp profiles/r04/fetch_sweep.txt gpurun_out/profiles/r04/
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_full.log
exit $rc
