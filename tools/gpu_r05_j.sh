#!/bin/bash
# Round 5, GPU call J: the bit-packed encoder kernel with in-place TB segments and the device CB CRC24B -- encoder,
# PDSCH plugin and C++ adapter tests first, then the whole -m gpu suite, extra.hal (PDSCH encoder slot figures), and a
# kernel trace of the HAL bench. Stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_encoder.py \
  tests/test_gpu_pdsch_enc.py -m gpu > gpurun_out/pytest_enc_r05j.txt 2>&1
rc=$?; tail -5 gpurun_out/pytest_enc_r05j.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r05j.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r05j.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/run_hal_bench.py 20 > gpurun_out/hal_r05j.json 2> gpurun_out/hal_r05j.log
rc=$?; echo "hal rc=$rc"; tail -c 700 gpurun_out/hal_r05j.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hal_r05j -o run -- python3 tools/run_hal_bench.py 5 > gpurun_out/prof_hal_r05j.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
