#!/bin/bash
# GPU box (round 6): the -m gpu suite and smoke(), then the committed evidence from this one build:
# tools/profile.sh (kernel trace + stats, PMC passes), tools/collect_profiles.py r06 (with profiles/fetch_fit.json of
# tools/fetch_sweep.sh), then the default bench line that reads the fresh pmc_traffic.json. Profile files come back
# under gpurun_out/profiles/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/smoke.txt; [ $rc -ne 0 ] && exit $rc
bash tools/profile.sh > gpurun_out/profile.txt 2>&1
rc=$?; cat gpurun_out/profile.txt; [ $rc -ne 0 ] && exit $rc
python3 tools/collect_profiles.py r06 gpurun_out/prof || exit 1
mkdir -p gpurun_out/profiles
cp profiles/pmc_traffic.json profiles/r06_kernel_stats.csv profiles/r06_pmc.txt gpurun_out/profiles/
timeout -k 10 600 python3 -u bench.py --extras-out gpurun_out/profiles/r06_bench_extras.json > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_full.log
tail -n 1 gpurun_out/bench_full.log > gpurun_out/profiles/r06_bench_line.json
exit $rc
