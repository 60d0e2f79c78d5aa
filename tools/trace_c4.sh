#!/bin/bash
# GPU box: kernel traces of replayed C4 slots, from symbols and from LLRs (tools/c4_trace.py [llrs]); timelines of
# the last dispatches by tools/trace_timeline.py. Output gpurun_out/pc4s, gpurun_out/pc4l.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc4s -o run -- python3 tools/c4_trace.py > gpurun_out/pc4s.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc4l -o run -- python3 tools/c4_trace.py llrs > gpurun_out/pc4l.log 2>&1 || exit 1
echo "== from symbols"; python3 tools/trace_timeline.py gpurun_out/pc4s 12
echo "== from LLRs"; python3 tools/trace_timeline.py gpurun_out/pc4l 12
