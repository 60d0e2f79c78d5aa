# GPU box: the whole -m gpu suite with the mid-size specialised kernels, then C3 and 128-CB batches of every
# specialised graph
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
L=srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip.so
timeout -k 10 180 python tools/time_c3.py $L > gpurun_out/g33_time.txt 2>&1 || exit 1
SW=1:384,1:352,1:320,1:288,1:256,1:240,1:224,1:208,1:192,1:176,1:160,1:144,1:128,2:384,2:352,2:320,2:288,2:256,2:240,2:224,2:208,2:192,2:176,2:160,2:144,2:128
timeout -k 10 300 python tools/time_variant.py $L sweep $SW >> gpurun_out/g33_time.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/g33_time.txt | cut -c1-200; exit $rc
