cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c4_full.py tests/test_gpu_tb_join.py -m gpu > gpurun_out/pytest_c4.log 2>&1
echo "rc=$?"; tail -12 gpurun_out/pytest_c4.log
