# GPU box: A/B of wave priority for the completing group in pipelined chain steps (prio) vs the product (cur)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
SW=1:384,1:320,1:256,2:384,2:208,2:128
: > gpurun_out/g38_time.txt
for rep in 1 2; do
  for v in cur prio; do
    timeout -k 10 120 python tools/time_variant.py $L/libsrsran_ldpc_hip_$v.so sweep $SW >> gpurun_out/g38_time.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/g38_time.txt
