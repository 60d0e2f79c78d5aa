cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decoder.py tests/test_gpu_c4_full.py -m gpu > gpurun_out/ab1_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab1_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_variants.sh ab1 2 1:384,1:352,1:320 base cur l0 || exit 1
for v in base cur l0; do f=$L/libsrsran_ldpc_hip_$v.so; [ $v = cur ] && f=$L/libsrsran_ldpc_hip.so; timeout -k 10 120 python tools/time_c4_lib.py $f 20 2>&1 | grep -v amdgpu.ids || exit 1; done
