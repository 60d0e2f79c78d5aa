#!/bin/bash
# Diagnostic: C2 kernel time (and 3-CB parity) of compiler-scheduling variants of the library, built with
#   make -C srsran_projectvtlmo_amd/csrc exp NAME=<v> FLAGS="-mllvm ..."
cd "$(dirname "$0")/.." || exit 1
for v in libsrsran_ldpc_hip.so libsrsran_ldpc_hip_ilp.so libsrsran_ldpc_hip_bias0.so libsrsran_ldpc_hip_bias100.so; do
  [ -f srsran_projectvtlmo_amd/lib/$v ] || continue
  timeout -k 10 120 python tools/time_variant.py srsran_projectvtlmo_amd/lib/$v || exit 1
done
