#!/bin/bash
# Round 5, GPU call F: binary16 soft bits in the specialised decoders -- the whole -m gpu suite on the product, then
# an A/B against the int8 build (-DLDPC_SPEC_F16=0, lib suffix i8): C2 and the Z sweep, alternating, two rounds.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_r05f_all.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/pytest_r05f_all.log
[ $rc -ne 0 ] && exit $rc
SWEEP="1:384,1:256,1:128,1:64,1:36,2:384,2:208,2:128,2:64,2:36,2:16"
LIBDIR=srsran_projectvtlmo_amd/lib
: > gpurun_out/ab_f16.txt
for r in 1 2; do
  for lib in libsrsran_ldpc_hip.so libsrsran_ldpc_hip_i8.so; do
    timeout -k 10 100 python -u tools/time_variant.py $LIBDIR/$lib >> gpurun_out/ab_f16.txt 2>&1 || exit 1
    timeout -k 10 200 python -u tools/time_variant.py $LIBDIR/$lib sweep $SWEEP >> gpurun_out/ab_f16.txt 2>&1 || exit 1
  done
done
echo "ab rc=0"; grep -v amdgpu.ids gpurun_out/ab_f16.txt | tail -26
