# GPU box: the whole -m gpu suite, a bench line (extras incl. z sweep and HAL), and the HAL-route trace
cd /root/repo && mkdir -p gpurun_out/prof_hal && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_quick.txt 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/write_slot_bin.py /tmp/slot.bin && \
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_hal -o run -- ./tests/cpp/build/bench_hal /tmp/slot.bin 3 > gpurun_out/prof_hal/trace.log 2>&1
rc=$?; echo "hal trace rc=$rc"; exit $rc
