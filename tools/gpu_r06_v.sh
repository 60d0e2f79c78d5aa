#!/bin/bash
# Round 6, call V: the HAL bench alternating the LDS-direct v3 library and the previous build, 3 rounds
set -o pipefail
mkdir -p gpurun_out
L=srsran_projectvtlmo_amd/lib
cp $L/libsrsran_ldpc_hip.so /tmp/new.so
for rep in 1 2 3; do
  for v in new pre; do
    if [ $v = new ]; then cp /tmp/new.so $L/libsrsran_ldpc_hip.so; else cp $L/libsrsran_ldpc_hip_r06pre.so $L/libsrsran_ldpc_hip.so; fi
    timeout -k 10 300 python3 -u tools/run_hal_bench.py > gpurun_out/r06v_hal_${v}_${rep}.json 2> gpurun_out/r06v_hal_${v}_${rep}.err || exit 1
  done
done
cp /tmp/new.so $L/libsrsran_ldpc_hip.so
