#!/bin/bash
# GPU-box driver script: parity tests, then a short bench. Stops after a crash/timeout/fault (exit 124/134/137/139).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) echo "stopping after GPU test failure mode $rc"; exit $rc;; esac
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -3 gpurun_out/bench.log
exit $(( rc != 0 ? rc : brc ))
