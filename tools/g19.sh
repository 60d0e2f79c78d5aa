# GPU box: HAL-route trace (kernels + memory copies) of bench_hal on the C4 slot
cd /root/repo && mkdir -p gpurun_out/prof_hal && export TMPDIR=/tmp
timeout -k 10 120 python tools/write_slot_bin.py /tmp/slot.bin && \
timeout -k 10 120 ./tests/cpp/build/bench_hal /tmp/slot.bin 20 > gpurun_out/prof_hal/bench_hal.json && \
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_hal -o run -- ./tests/cpp/build/bench_hal /tmp/slot.bin 3 > gpurun_out/prof_hal/trace.log 2>&1
rc=$?; echo rc=$rc; cat gpurun_out/prof_hal/bench_hal.json; exit $rc
