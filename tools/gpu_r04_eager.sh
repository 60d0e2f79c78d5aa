#!/bin/bash
# GPU box (round 4): enqueue-time HAL submission + post-item polls -- the work-queue and HAL suites, the full -m gpu
# suite, then the routes A/B: product (32 workgroups per queue, enqueue-time HAL submission), without it
# (LDPC_HIP_HAL_EAGER=0), 64 workgroups, and the mirror-based protocol (variant dwqold).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dwq.py tests/test_gpu_hal.py -x -q --timeout 60 --timeout-method thread > gpurun_out/pytest_hal.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_hal.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u tools/route_ab.py 2 new noeager:LDPC_HIP_HAL_EAGER=0 wg64:LDPC_HIP_DWQ_WORKGROUPS=64 old:LIB=dwqold > gpurun_out/route_ab3.json 2> gpurun_out/route_ab3.log
rc=$?; tail -c 3000 gpurun_out/route_ab3.log; exit $rc
