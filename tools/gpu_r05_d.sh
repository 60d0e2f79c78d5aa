#!/bin/bash
# Round 5, GPU call D: the register-resident decoder of the one-wave graphs (Z <= 64) -- decoder / work-queue / HAL /
# slot suites, then an A/B of the product library against the lane-split build (-DLDPC_SPEC_REG=0, lib suffix quad)
# over the one-wave graphs, alternating, two rounds. Stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decoder.py \
  tests/test_gpu_dwq.py tests/test_gpu_hal.py tests/test_gpu_c4_full.py tests/test_gpu_slot.py -m gpu \
  > gpurun_out/pytest_r05d_core.log 2>&1
rc=$?; echo "core tests rc=$rc"; tail -5 gpurun_out/pytest_r05d_core.log
[ $rc -ne 0 ] && exit $rc
SWEEP="1:2,1:8,1:16,1:24,1:32,1:36,1:48,1:64,2:2,2:8,2:16,2:24,2:32,2:36,2:48,2:64"
LIBDIR=srsran_projectvtlmo_amd/lib
: > gpurun_out/ab_reg.txt
for r in 1 2; do
  for lib in libsrsran_ldpc_hip.so libsrsran_ldpc_hip_quad.so; do
    timeout -k 10 200 python -u tools/time_variant.py $LIBDIR/$lib sweep $SWEEP >> gpurun_out/ab_reg.txt 2>&1 || exit 1
    timeout -k 10 100 python -u tools/time_variant.py $LIBDIR/$lib 2 36 1 1 >> gpurun_out/ab_reg.txt 2>&1 || exit 1
    timeout -k 10 100 python -u tools/time_variant.py $LIBDIR/$lib 1 52 2 1 >> gpurun_out/ab_reg.txt 2>&1 || exit 1
  done
done
echo "ab rc=0"; grep -v amdgpu.ids gpurun_out/ab_reg.txt | tail -40
