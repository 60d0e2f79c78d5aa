#!/bin/bash
# GPU box (round 4): the -m gpu suite on the product library, the small-Z A/B of single rows split on one-wave graphs
# (variants t4 / t6: LDPC_SPEC_SPLIT_TINY = 4 / 6 against the product's 12), and the software-route / HAL A/B with
# and without the device work queue (tools/sw_route_ab.py). Output under gpurun_out/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
bash tools/ab_variants.sh small_z 2 "1:64,2:64,1:52,2:52,1:36,2:36,1:16,2:16,1:2,2:2" cur t4 t6 || exit 1
timeout -k 10 600 python -u tools/sw_route_ab.py 10 1,4,8,16 > gpurun_out/sw_route_ab.txt 2>&1
rc=$?; tail -c 600 gpurun_out/sw_route_ab.txt; exit $rc
