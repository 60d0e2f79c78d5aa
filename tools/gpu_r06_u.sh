#!/bin/bash
# Round 6, call U: LDS-direct fused dematch v3 (LDS-only writes, stash flushed after the prologue):
# every dematch-touching suite on the new library, then the HAL bench and the C4 slot alternating the new library and
# the previous build (libsrsran_ldpc_hip_r06pre.so swapped in under the product name), 2 rounds
set -o pipefail
mkdir -p gpurun_out
L=srsran_projectvtlmo_amd/lib
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rm_reference_table.py tests/test_gpu_dwq.py tests/test_gpu_hal.py tests/test_gpu_hal_cases.py tests/test_gpu_slot.py tests/test_gpu_c4_full.py tests/test_gpu_demod.py tests/test_gpu_cpp_adapters.py > gpurun_out/r06u_pytest.txt 2>&1 || exit 1
cp $L/libsrsran_ldpc_hip.so /tmp/new.so
for rep in 1 2; do
  for v in new pre; do
    if [ $v = new ]; then cp /tmp/new.so $L/libsrsran_ldpc_hip.so; else cp $L/libsrsran_ldpc_hip_r06pre.so $L/libsrsran_ldpc_hip.so; fi
    timeout -k 10 300 python3 -u tools/run_hal_bench.py > gpurun_out/r06u_hal_${v}_${rep}.json 2> gpurun_out/r06u_hal_${v}_${rep}.err || exit 1
    timeout -k 10 200 python3 -u tools/time_c4_lib.py $L/libsrsran_ldpc_hip.so 20 >> gpurun_out/r06u_c4.txt 2>&1 || exit 1
    echo "== $v $rep" >> gpurun_out/r06u_c4.txt
  done
done
cp /tmp/new.so $L/libsrsran_ldpc_hip.so
