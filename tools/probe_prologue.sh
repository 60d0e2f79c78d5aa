#!/bin/bash
# GPU box: prologue probes: time_et.py (all-zero codeword, one iteration; all-zero LLRs) on the product and on the
# timing-only build without the split-address table fill (nofill).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
for v in cur nofill cur nofill; do f=$L/libsrsran_ldpc_hip_$v.so; [ $v = cur ] && f=$L/libsrsran_ldpc_hip.so
  echo "== $v"; timeout -k 10 200 python tools/time_et.py $f 2>&1 | grep -v amdgpu.ids | head -6 || exit 1; done
