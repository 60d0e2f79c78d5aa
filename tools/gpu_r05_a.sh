#!/bin/bash
# Round 5, GPU call A: the new stream / work-queue / HAL tests first, then the whole -m gpu suite, a quick bench
# (extras on: sw_route with its CPU leg and the "auto" pairing), then the stream-handle probe for hipStreamLegacy
# (last: it may crash in the runtime, which is what it is there to show). Stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_streams.py \
  tests/test_gpu_dwq.py tests/test_gpu_hal.py tests/test_gpu_cpp_adapters.py -m gpu > gpurun_out/pytest_r05a_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -5 gpurun_out/pytest_r05a_new.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_r05a_all.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/pytest_r05a_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --steps 50 --warmup 5 --cpu-baseline auto --cpu-reps 300 \
  > gpurun_out/bench_r05a.txt 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 gpurun_out/bench_r05a.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 60 tools/ubench/stream_probe 1 > gpurun_out/stream_probe_legacy.txt 2>&1
rc=$?; echo "probe legacy rc=$rc"; cat gpurun_out/stream_probe_legacy.txt
exit $rc
