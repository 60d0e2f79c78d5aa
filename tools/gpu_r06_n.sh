#!/bin/bash
# Round 6, call N: LDS-direct fused dematch on the work queue. (1) the work-queue, HAL (incl. the 174-case table),
# slot and C++ adapter suites on the new library; (2) the HAL bench (C4 slot through the plugin), alternating the new
# library and the round's previous build (libsrsran_ldpc_hip_r06pre.so swapped in under the product name), 2 rounds
set -o pipefail
mkdir -p gpurun_out
L=srsran_projectvtlmo_amd/lib
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dwq_timeout.py tests/test_gpu_dwq.py tests/test_gpu_hal.py tests/test_gpu_hal_cases.py tests/test_gpu_slot.py tests/test_gpu_cpp_adapters.py > gpurun_out/r06n_pytest.txt 2>&1 || exit 1
cp $L/libsrsran_ldpc_hip.so /tmp/new.so
for rep in 1 2; do
  for v in new pre; do
    if [ $v = new ]; then cp /tmp/new.so $L/libsrsran_ldpc_hip.so; else cp $L/libsrsran_ldpc_hip_r06pre.so $L/libsrsran_ldpc_hip.so; fi
    timeout -k 10 300 python3 -u tools/run_hal_bench.py > gpurun_out/r06n_hal_${v}_${rep}.json 2> gpurun_out/r06n_hal_${v}_${rep}.err || exit 1
  done
done
cp /tmp/new.so $L/libsrsran_ldpc_hip.so
