cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hal.py tests/test_gpu_cpp_adapters.py tests/test_gpu_decoder.py -m gpu > gpurun_out/pytest_hal.log 2>&1
echo "rc=$?"; tail -5 gpurun_out/pytest_hal.log
