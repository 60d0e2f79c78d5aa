#!/bin/bash
# Round 6, call C: kernel trace of C2 beside 0 / 4 idle work-queue grids (per-kernel durations and inter-kernel gaps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06c
export LDPC_HIP_DWQ_IDLE_US=1000000
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r06c/g0 -o g0 -- python3 $R/tools/dwq_tax_ab.py child 0 idle > $R/gpurun_out/r06c/g0.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r06c/g4 -o g4 -- python3 $R/tools/dwq_tax_ab.py child 4 idle > $R/gpurun_out/r06c/g4.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r06c/g1 -o g1 -- python3 $R/tools/dwq_tax_ab.py child 1 idle > $R/gpurun_out/r06c/g1.log 2>&1
