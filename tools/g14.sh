cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench/sem16 > gpurun_out/sem16.txt 2>&1; cat gpurun_out/sem16.txt
bash tools/run_variants.sh _w32 "" _w32 "" && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_c4_full.py -m gpu > gpurun_out/pytest_dec.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_dec.log; exit $rc
