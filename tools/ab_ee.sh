#!/bin/bash
# GPU box: skipped barriers of empty steps (product) vs every step's barrier (ee0): decoder parity tests, C2-size
# batches and the C4 slot (ab_c2_c4.sh), and the fixed/per-iteration costs (time_et.py) of both libraries.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_c4_full.py tests/test_gpu_slot.py -m gpu > gpurun_out/ee_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ee_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_c2_c4.sh ab3 1:384,1:256,2:208,2:36 cur ee0 || exit 1
for v in ee0 cur; do f=srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip_$v.so; [ $v = cur ] && f=srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip.so
  echo "== $v"; timeout -k 10 200 python tools/time_et.py $f 2>&1 | grep -v amdgpu.ids || exit 1; done
