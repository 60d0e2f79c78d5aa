#!/bin/bash
# Round 5, GPU call O: the PDSCH rate matcher stages its bytes in LDS and stores 16 bytes at a time; AVX2 bit unpack in the dequeue -- encoder,
# PDSCH plugin and C++ adapter tests first, then the whole -m gpu suite, extra.hal (PDSCH encoder slot figures), and a
# kernel trace of the HAL bench. Stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_encoder.py \
  tests/test_gpu_pdsch_enc.py tests/test_gpu_cpp_adapters.py -m gpu > gpurun_out/pytest_enc_r05o.txt 2>&1
rc=$?; tail -5 gpurun_out/pytest_enc_r05o.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r05o.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r05o.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/run_hal_bench.py 20 > gpurun_out/hal_r05o.json 2> gpurun_out/hal_r05o.log
rc=$?; echo "hal rc=$rc"; tail -c 700 gpurun_out/hal_r05o.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/hal_blob.py gpurun_out/slot_r05o.bin || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hal_r05o -o run -- tests/cpp/build/bench_hal gpurun_out/slot_r05o.bin 5 0 > gpurun_out/prof_hal_r05o.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
