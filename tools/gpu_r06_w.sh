#!/bin/bash
# GPU box (round 6): the -m gpu suite on the system-coherent pinned-LLR loads (host_load16), then the host-memory
# routes A/B against the previous build (tools/route_ab.py: libsrsran_ldpc_hip_before.so vs _hostld.so).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_w.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_w.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u tools/route_ab.py 3 before:LIB=before hostld:LIB=hostld > gpurun_out/r06w_route_ab.json 2> gpurun_out/r06w_route_ab.err
rc=$?; tail -c 600 gpurun_out/r06w_route_ab.err; exit $rc
