#!/bin/bash
# GPU box: split-step cost probes (timing-only builds, wrong results): tools/time_split.py per library, two rounds.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
for rep in 1 2; do for v in cur nomerge nowrite noread norw ee0; do
  f=$L/libsrsran_ldpc_hip_$v.so; [ $v = cur ] && f=$L/libsrsran_ldpc_hip.so
  timeout -k 10 120 python tools/time_split.py $f 2>&1 | grep -v amdgpu.ids || exit 1
done; done
