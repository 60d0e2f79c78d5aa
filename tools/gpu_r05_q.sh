#!/bin/bash
# Round 5, GPU call Q: kernel trace of the HAL bench with the copy work queue on (LDPC_HIP_HAL_DWQ_COPY=1): where the
# 128-CB TB's first dequeue goes (copy items, then the batch kernel reading HBM).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python3 tools/hal_blob.py gpurun_out/slot_r05q.bin || exit 1
LDPC_HIP_HAL_DWQ_COPY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hal_r05q -o run -- tests/cpp/build/bench_hal gpurun_out/slot_r05q.bin 5 0 > gpurun_out/prof_hal_r05q.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
