#!/bin/bash
# GPU box (round 6): the -m gpu suite with the one-CB decode's LLRs staged in BAR-written device memory
# (ldpc_hip_buffers.h bar_buffer), then the host-memory routes A/B against the pinned staging
# (LDPC_HIP_BAR_STAGING=0) on the same library (tools/route_ab.py, three alternating rounds).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_bar.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_bar.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 -u tools/route_ab.py 3 pinned:LDPC_HIP_BAR_STAGING=0 bar:LDPC_HIP_BAR_STAGING=1 > gpurun_out/r06bar_route_ab.json 2> gpurun_out/r06bar_route_ab.err
rc=$?; tail -c 300 gpurun_out/r06bar_route_ab.err; exit $rc
