# GPU box: pipelined single-row chains -- A/B timing vs HEAD and the no-pipeline build, then the decoder parity tests
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
SW=1:384,1:352,1:320,1:288,1:256,2:384,2:352,2:320,2:288,2:256
for rep in 1 2; do
  for v in base nopipe ""; do
    f=$L/libsrsran_ldpc_hip${v:+_$v}.so
    timeout -k 10 120 python tools/time_variant.py $f sweep $SW >> gpurun_out/g27_time.txt 2>&1 || exit 1
  done
done
cat gpurun_out/g27_time.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py > gpurun_out/g27_tests.log 2>&1
rc=$?; tail -5 gpurun_out/g27_tests.log; exit $rc
