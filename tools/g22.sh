cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_multi_cell.py tests/test_gpu_cpp_adapters.py tests/test_gpu_decoder.py -m gpu > gpurun_out/pytest_mc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_mc.log; exit $rc
