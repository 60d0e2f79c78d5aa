#!/bin/bash
# GPU box (round 4): the slot-polling work queue -- its parity suites first (work queue, HAL, software route), the
# full -m gpu suite, then the host-memory routes A/B against the previous protocol (variant dwqold).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dwq.py -x -q --timeout 60 --timeout-method thread > gpurun_out/pytest_dwq.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_dwq.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u tools/route_ab.py 2 new old:LIB=dwqold > gpurun_out/route_ab2.json 2> gpurun_out/route_ab2.log
rc=$?; tail -c 1500 gpurun_out/route_ab2.log; exit $rc
