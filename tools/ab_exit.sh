#!/bin/bash
# GPU box: A/B of the product decoder library against variants (default: head = the previous commit's build):
# decoder/C4/slot/HAL parity tests on the product, the 4/6-layer iteration cost (time_split.py), the early-stop
# check cost and the per-CB fixed cost (time_et.py), C3 (time_c3.py), 128-CB batches and the C4 slot (ab_c2_c4.sh, two rounds).
# Usage: ab_exit.sh OUT [variant...]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=${1:-ab}; shift; VARS=${*:-head}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_c4_full.py tests/test_gpu_slot.py tests/test_gpu_hal.py -m gpu > gpurun_out/exit_tests.log 2>&1
rc=$?; tail -2 gpurun_out/exit_tests.log; [ $rc -ne 0 ] && exit $rc
L=srsran_projectvtlmo_amd/lib
for v in $VARS cur; do f=$L/libsrsran_ldpc_hip_$v.so; [ $v = cur ] && f=$L/libsrsran_ldpc_hip.so
  echo "== $v"
  timeout -k 10 120 python tools/time_split.py $f 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python tools/time_et.py $f 2>&1 | grep -v amdgpu.ids | head -4 || exit 1
  timeout -k 10 120 python tools/time_et.py $f rounds 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 120 python tools/time_c3.py $f 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/ab_c2_c4.sh "$OUT" 1:384,1:352,1:256,1:128,2:208,2:36 $VARS cur
