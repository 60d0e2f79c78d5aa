# GPU box: the whole -m gpu suite with the mid-size specialised kernels, then C3 and 128-CB batches of every
# specialised graph
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
L=srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip.so
: > gpurun_out/g33_time.txt
SW=1:120,1:112,1:104,1:96,1:88,1:80,1:72,1:64,2:120,2:112,2:104,2:96,2:88,2:80,2:72,2:64
timeout -k 10 300 python tools/time_variant.py $L sweep $SW >> gpurun_out/g33_time.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/g33_time.txt | cut -c1-200; exit $rc
