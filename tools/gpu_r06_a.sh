#!/bin/bash
# Round 6, call A: the new bench line format, the DWQ tax A/B, the work-queue tests (stop-claims-nothing, timeout path)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dwq_timeout.py tests/test_gpu_dwq.py > gpurun_out/r06a_pytest_dwq.txt 2>&1 &&
timeout -k 10 400 python3 -u bench.py > gpurun_out/r06a_bench.log 2> gpurun_out/r06a_bench.err &&
timeout -k 10 500 python3 -u tools/dwq_tax_ab.py > gpurun_out/r06a_tax.log 2>&1
