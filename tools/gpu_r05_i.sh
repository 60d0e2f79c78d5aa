#!/bin/bash
# Round 5, GPU call I (re-entry after the container was re-created): the -m gpu suite and smoke() on the rebuilt
# tree, then extra.hal alone (HAL decoder and PDSCH encoder slot figures) as the baseline for the encoder work.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r05i.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r05i.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05i.txt 2>&1
rc=$?; tail -2 gpurun_out/smoke_r05i.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/run_hal_bench.py 20 > gpurun_out/hal_r05i.json 2> gpurun_out/hal_r05i.log
rc=$?; echo "hal rc=$rc"; tail -c 1500 gpurun_out/hal_r05i.json
exit $rc
