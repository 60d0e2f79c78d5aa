#!/bin/bash
# GPU box (round 4): tools/diag_dwq.py on the LDPC_HIP_DIAG_DWQ + LDPC_HIP_DIAG_CB build (where a one-CB call's time
# goes), then the -m gpu suite on the product library. Output under gpurun_out/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/diag_dwq.py 200 > gpurun_out/diag_dwq.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/diag_dwq.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; exit $rc
