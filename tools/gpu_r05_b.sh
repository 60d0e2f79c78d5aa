#!/bin/bash
# Round 5, GPU call B: the lane-split small-Z decoder (sp::qdec) -- decoder / work-queue / HAL / slot suites, then
# the whole -m gpu suite, a quick bench (z_sweep, HAL, software route), the diagnostic timelines (C2's BG1 Z=384 and
# the previous BG2 Z=36 kernel, from the diag libraries built before the change), the work-queue residency A/B and
# the HAL early-copy A/B. Each step under its own time limit; stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decoder.py \
  tests/test_gpu_dwq.py tests/test_gpu_hal.py tests/test_gpu_c4_full.py tests/test_gpu_slot.py -m gpu \
  > gpurun_out/pytest_r05b_core.log 2>&1
rc=$?; echo "core tests rc=$rc"; tail -5 gpurun_out/pytest_r05b_core.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_r05b_all.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/pytest_r05b_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --cpu-baseline off > gpurun_out/bench_r05b.txt 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 200 gpurun_out/bench_r05b.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/diag_timeline.py 1 384 8 diagfull > gpurun_out/timeline_c2_diagfull.txt 2>&1 && \
timeout -k 10 120 python -u tools/diag_timeline.py 1 384 8 diag > gpurun_out/timeline_c2_diag.txt 2>&1 && \
timeout -k 10 120 python -u tools/diag_timeline.py 2 36 8 diagfull m > gpurun_out/timeline_bg2z36_old_diagfull.txt 2>&1
rc=$?; echo "timelines rc=$rc"; tail -4 gpurun_out/timeline_c2_diagfull.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/dwq_residency_ab.py > gpurun_out/dwq_residency_ab.txt 2>&1
rc=$?; echo "residency rc=$rc"; tail -c 600 gpurun_out/dwq_residency_ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/route_ab.py 2 base early:LDPC_HIP_HAL_EARLY_COPY=1 \
  early64k:LDPC_HIP_HAL_EARLY_COPY=1,LDPC_HIP_HAL_COPY_CHUNK=65536 > gpurun_out/route_ab_early_copy.json 2>&1
rc=$?; echo "route_ab rc=$rc"
exit $rc
