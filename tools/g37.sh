# GPU box: kernel + memory-copy trace of the HAL route (bench_hal on the C4 slot, 3 reps)
cd /root/repo && mkdir -p gpurun_out/phal && export TMPDIR=/tmp
timeout -k 10 120 python tools/write_slot_bin.py /tmp/slot.bin || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/phal -o run -- tests/cpp/build/bench_hal /tmp/slot.bin 3 > gpurun_out/phal/hal.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
