#!/bin/bash
# Diagnostic: generic-decoder kernel time for BG2 Z=208 batches (C3 shape) wide (LDPC_HIP_NARROW=0) vs narrow (=1) schedules.
L=srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip.so
for nw in 0 1; do
  for a in "2 208 1 256" "2 208 1 1024" "2 208 10 1024"; do
    LDPC_HIP_NARROW=$nw timeout -k 10 120 python tools/time_variant.py $L $a || exit 1
  done
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/bench_c4.log 2>&1
