#!/bin/bash
# Diagnostic: rocprofv3 kernel trace of the whole bench (C2 + C3/C4 extras) -> gpurun_out/px; summarised by
# tools/trace_summary.py (per-kernel average durations).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/px
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/px -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/px/b.log 2>&1
