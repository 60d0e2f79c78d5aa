#!/bin/bash
# GPU box: A/B timing of decoder library variants against each other (diagnostic, not product).
#
#   ab_variants.sh OUT ROUNDS SWEEP SUFFIX...
#
# Each SUFFIX names srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip_<SUFFIX>.so ("cur" or "" = the product library),
# built beforehand on the CPU with  make -C srsran_projectvtlmo_amd/csrc exp NAME=<SUFFIX> FLAGS="-D..."  .
# SWEEP is tools/time_variant.py's graph list (bg:Z,bg:Z,...; 128 CBs, 8 iterations, parity vs the product checked on
# three CBs). The variants alternate ROUNDS times on one box, so box-to-box drift cancels. Output: gpurun_out/OUT.txt.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/$1.txt; ROUNDS=$2; SWEEP=$3; shift 3
L=srsran_projectvtlmo_amd/lib
: > "$OUT"
for rep in $(seq "$ROUNDS"); do
  for v in "$@"; do
    case $v in cur|"") f=$L/libsrsran_ldpc_hip.so ;; *) f=$L/libsrsran_ldpc_hip_$v.so ;; esac
    timeout -k 10 120 python tools/time_variant.py "$f" sweep "$SWEEP" >> "$OUT" 2>&1 || exit 1
  done
done
grep -v amdgpu.ids "$OUT"
