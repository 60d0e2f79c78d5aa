#!/bin/bash
# GPU box: early-stop check composition probes (timing-only builds): time_et.py's all-zero-codeword cases per library.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
for v in cur nocrc nomul nohd; do f=$L/libsrsran_ldpc_hip_$v.so; [ $v = cur ] && f=$L/libsrsran_ldpc_hip.so
  echo "== $v"; timeout -k 10 200 python tools/time_et.py $f 2>&1 | grep -v amdgpu.ids | head -4 || exit 1; done
