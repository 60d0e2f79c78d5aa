#!/bin/bash
# Round 5, GPU call E: the register-resident decoder without per-row scheduling barriers, timed over the one-wave
# graphs (parity of the first CBs checked by time_variant.py), two rounds.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
SWEEP="1:2,1:8,1:16,1:24,1:32,1:36,1:48,1:64,2:2,2:8,2:16,2:24,2:32,2:36,2:48,2:64"
LIBDIR=srsran_projectvtlmo_amd/lib
: > gpurun_out/ab_reg_e.txt
for r in 1 2; do
  for lib in libsrsran_ldpc_hip.so; do
    timeout -k 10 200 python -u tools/time_variant.py $LIBDIR/$lib sweep $SWEEP >> gpurun_out/ab_reg_e.txt 2>&1 || exit 1
    timeout -k 10 100 python -u tools/time_variant.py $LIBDIR/$lib 2 36 1 1 >> gpurun_out/ab_reg_e.txt 2>&1 || exit 1
  done
done
echo "ab rc=0"; grep -v amdgpu.ids gpurun_out/ab_reg_e.txt | tail -20
