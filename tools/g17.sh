cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pdsch_enc.py tests/test_gpu_cpp_adapters.py -m gpu > gpurun_out/pytest_enc.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_enc.log | tail -30; exit $rc
