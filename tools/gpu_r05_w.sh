#!/bin/bash
# Round 5, GPU call W: the driver's round-end checks at HEAD -- the whole -m gpu suite and smoke().
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r05w.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r05w.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05w.txt 2>&1
rc=$?; tail -2 gpurun_out/smoke_r05w.txt; exit $rc
