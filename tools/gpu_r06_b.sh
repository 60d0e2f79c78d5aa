#!/bin/bash
# Round 6, call B: CU placement / full-chip A/B for the work-queue tax, and the C++ adapter test (auto split)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 tests/cpp/build/test_adapters > gpurun_out/r06b_cpp.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/cu_placement_ab.py > gpurun_out/r06b_cu.log 2>&1
