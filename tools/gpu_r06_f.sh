#!/bin/bash
# Round 6, call F: work-queue pool capped at 2 hardware queues + pinned admission: the work-queue tests, HAL and
# PDSCH suites, the C++ adapters, the tax A/B and the bench (HAL / software-route extras)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dwq_timeout.py tests/test_gpu_dwq.py tests/test_gpu_hal.py tests/test_gpu_hal_cases.py tests/test_gpu_pdsch_enc.py tests/test_gpu_cpp_adapters.py > gpurun_out/r06f_pytest.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/dwq_tax_ab.py none g1_idle g4_idle g4_items > gpurun_out/r06f_tax.log 2>&1 &&
timeout -k 10 400 python3 -u bench.py --extras-out gpurun_out/r06f_extras.json > gpurun_out/r06f_bench.log 2> gpurun_out/r06f_bench.err
