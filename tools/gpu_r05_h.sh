#!/bin/bash
# Round 5, GPU call H: the lane-split address table kept in registers across work-queue items -- decoder /
# work-queue / HAL / slot suites on the product, one-CB phases (tools/diag_dwq.py, diagdwq build), then the
# host-memory routes against the previous library (r05a), alternating, three rounds. Stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decoder.py \
  tests/test_gpu_dwq.py tests/test_gpu_hal.py tests/test_gpu_hal_cases.py tests/test_gpu_c4_full.py \
  tests/test_gpu_slot.py -m gpu > gpurun_out/pytest_r05h_core.log 2>&1
rc=$?; echo "core tests rc=$rc"; tail -3 gpurun_out/pytest_r05h_core.log
[ $rc -ne 0 ] && exit $rc
DIAG_LIB=diagdwq timeout -k 10 300 python3 -u tools/diag_dwq.py 200 > gpurun_out/diag_dwq_r05h.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/diag_dwq_r05h.txt | grep "BG\|body\|outside\|entry -> done"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/route_ab.py 3 product old:LIB=r05a > gpurun_out/route_ab_qpre.json 2> gpurun_out/route_ab_qpre.log
rc=$?; echo "route_ab rc=$rc"; tail -c 1500 gpurun_out/route_ab_qpre.json
exit $rc
