# GPU box: the whole -m gpu suite, then a kernel trace of replayed C4 slots (TB join timing)
cd /root/repo && mkdir -p gpurun_out/pc4 && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc4 -o run -- python3 tools/c4_trace.py > gpurun_out/pc4/c4.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
