#!/bin/bash
# Round 5, GPU call S: the PDSCH plugin's small-batch routes (work queue and launch) in both modes, against the oracle.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pdsch_enc.py -m gpu > gpurun_out/pytest_pdsch_r05s.txt 2>&1
rc=$?; tail -16 gpurun_out/pytest_pdsch_r05s.txt; exit $rc
