#!/bin/bash
# GPU box: the work-queue and HAL suites, the full -m gpu suite, the host-memory routes A/B of the product against
# the library variants named in the arguments (tools/route_ab.py configurations, e.g. "old:LIB=pg1"), and where a
# one-CB call's time goes (tools/diag_dwq.py on the diagdwq build, when it exists). Output under gpurun_out/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dwq.py tests/test_gpu_hal.py -x -q --timeout 60 --timeout-method thread > gpurun_out/pytest_hal.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_hal.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 480 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u tools/route_ab.py ${ROUNDS:-2} product "$@" > gpurun_out/route_ab.json 2> gpurun_out/route_ab.log
rc=$?; tail -c 2500 gpurun_out/route_ab.log; [ $rc -ne 0 ] && exit $rc
if [ -f srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip_diagdwq.so ]; then
  timeout -k 10 300 python3 -u tools/diag_dwq.py 200 > gpurun_out/diag_dwq.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/diag_dwq.txt; [ $rc -ne 0 ] && exit $rc
fi
exit 0
