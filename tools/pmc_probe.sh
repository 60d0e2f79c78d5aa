#!/bin/bash
# GPU-box: list the available counters, then one PMC pass of instruction-cache and VALU counters over a short C2 bench.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcp
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmcp/counters.txt 2>&1
B="bench.py --steps 5 --warmup 1 --cpu-baseline off --extras off"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmcp/p1 -o run -- python3 $B > gpurun_out/pmcp/p1.log 2>&1
echo "p1 rc=$?"
