#!/bin/bash
# Round 5, GPU call P: the HAL decoder's early copy of a large batch through copy work-queue items
# (LDPC_HIP_HAL_DWQ_COPY, ldpc_dwq_copy_kernel) -- HAL, work-queue and slot suites, the whole -m gpu suite, then
# extra.hal with the copy queue off / on, alternating, two rounds, and a kernel trace of the HAL bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
LDPC_HIP_HAL_DWQ_COPY=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hal.py \
  tests/test_gpu_hal_cases.py tests/test_gpu_dwq.py tests/test_gpu_cpp_adapters.py -m gpu > gpurun_out/pytest_hal_r05p.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_hal_r05p.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r05p.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r05p.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 0 1; do
    LDPC_HIP_HAL_DWQ_COPY=$v timeout -k 10 300 python3 -u tools/run_hal_bench.py 20 > gpurun_out/hal_r05p_c${v}_$r.json 2> gpurun_out/hal_r05p_c${v}_$r.log
    rc=$?; echo "copy=$v round $r rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 -c "import json,sys; d=json.load(open('gpurun_out/hal_r05p_c${v}_$r.json')); print(d['pusch_dec']['slot_us_p50'], d['pusch_dec_phases_us_p50']['multi_cb_tb'], {k: v['slot_us_p50'] for k, v in d['pusch_dec_concurrent'].items()})"
  done
done
timeout -k 10 120 python3 tools/hal_blob.py gpurun_out/slot_r05p.bin || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hal_r05p -o run -- tests/cpp/build/bench_hal gpurun_out/slot_r05p.bin 5 0 > gpurun_out/prof_hal_r05p.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
