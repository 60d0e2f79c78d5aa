#!/bin/bash
# GPU box: A/B of library variants on 128-CB batches (ab_variants.sh, two rounds) and on the C4 slot
# (time_c4_lib.py). Usage: ab_c2_c4.sh OUT SWEEP SUFFIX...   (suffix cur = the product library)
cd "$(dirname "$0")/.." || exit 1
OUT=$1; SWEEP=$2; shift 2
bash tools/ab_variants.sh "$OUT" 2 "$SWEEP" "$@" || exit 1
L=srsran_projectvtlmo_amd/lib
for v in "$@"; do
  f=$L/libsrsran_ldpc_hip_$v.so; [ "$v" = cur ] && f=$L/libsrsran_ldpc_hip.so
  timeout -k 10 120 python tools/time_c4_lib.py "$f" 20 2>&1 | grep -v amdgpu.ids | tee -a "gpurun_out/$OUT.txt" || exit 1
done
