#!/bin/bash
# GPU box: the whole -m gpu suite, smoke(), then a short bench without the CPU baseline. Each GPU step under its own
# time limit; stops at the first failure. Logs under gpurun_out/ (read them after the call).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --cpu-baseline off ${BENCH_ARGS:-} \
  > gpurun_out/bench_quick.txt 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_quick.txt
exit $rc
