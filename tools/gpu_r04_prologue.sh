#!/bin/bash
# GPU box (round 4): parity of the product after the any-alignment prologue and dematch staging changes (-m gpu), the
# small-Z batch times, and the host-memory routes A/B: product, HAL zero-copy up to 4 MiB, fast-poll work queue.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
bash tools/ab_variants.sh small_z_prologue 1 "2:36,1:36,2:52,1:52,2:64,1:64,2:16,2:13,1:13" cur || exit 1
timeout -k 10 900 python3 -u tools/route_ab.py 2 base zc4m:LDPC_HIP_HAL_ZERO_COPY_MAX=4194304 fast:LIB=dwqfast > gpurun_out/route_ab.json 2> gpurun_out/route_ab.log
rc=$?; tail -c 1500 gpurun_out/route_ab.log; exit $rc
