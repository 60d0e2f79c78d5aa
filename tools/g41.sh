# GPU box: occupancy A/B for the mid specialised kernels (amdgpu_waves_per_eu 6 / 8, with spills) vs the product:
# C3 decomposition, 1024-CB batches of BG1/BG2 Z=208, and 128-CB batches of mid graphs.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
: > gpurun_out/g41_time.txt
for v in cur wpe6 wpe8; do
  echo "== $v" >> gpurun_out/g41_time.txt
  timeout -k 10 120 python tools/c3_decomp.py $L/libsrsran_ldpc_hip_$v.so >> gpurun_out/g41_time.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/time_variant.py $L/libsrsran_ldpc_hip_$v.so 2 208 8 1024 >> gpurun_out/g41_time.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/time_variant.py $L/libsrsran_ldpc_hip_$v.so 1 208 8 1024 >> gpurun_out/g41_time.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/time_variant.py $L/libsrsran_ldpc_hip_$v.so sweep 1:240,1:208,1:128,2:208,2:128,2:64 >> gpurun_out/g41_time.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/g41_time.txt
