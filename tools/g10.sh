cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py -m gpu > gpurun_out/pytest_dec.log 2>&1
echo "pytest rc=$?"; tail -15 gpurun_out/pytest_dec.log
timeout -k 10 120 python tools/time_variant.py srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip.so 2>&1 | grep median
