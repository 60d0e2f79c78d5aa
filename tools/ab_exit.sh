#!/bin/bash
# GPU box: A/B of the decoder library against the previous commit (head): decoder
# parity tests on the product, the 4/6-layer iteration cost (time_split.py), 128-CB batches and the C4 slot.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_c4_full.py tests/test_gpu_slot.py tests/test_gpu_hal.py -m gpu > gpurun_out/exit_tests.log 2>&1
rc=$?; tail -2 gpurun_out/exit_tests.log; [ $rc -ne 0 ] && exit $rc
L=srsran_projectvtlmo_amd/lib
for v in head cur; do f=$L/libsrsran_ldpc_hip_$v.so; [ $v = cur ] && f=$L/libsrsran_ldpc_hip.so
  timeout -k 10 120 python tools/time_split.py $f 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/ab_c2_c4.sh ab9 1:384,1:352,1:256,1:128,2:208,2:36 head cur
