#!/bin/bash
# Round 5, first GPU call: a quick bench at HEAD (baseline for the round), then the special-stream-handle probe
# (tools/ubench/stream_probe.hip) for hipStreamPerThread, then hipStreamLegacy (the handle that segfaulted in round 4),
# each under its own time limit; stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --cpu-baseline off > gpurun_out/bench_quick_r05_head.txt 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_quick_r05_head.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 60 tools/ubench/stream_probe 2 > gpurun_out/stream_probe_perthread.txt 2>&1
rc=$?; echo "probe perthread rc=$rc"; cat gpurun_out/stream_probe_perthread.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 60 tools/ubench/stream_probe 1 > gpurun_out/stream_probe_legacy.txt 2>&1
rc=$?; echo "probe legacy rc=$rc"; cat gpurun_out/stream_probe_legacy.txt
exit $rc
