# GPU box: A/B of wave priority on BG1 graphs with W = 2 (pw2) against the product (cur: W >= 3 only); two rounds.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
SW=1:128,1:112,1:96,1:80,1:72,1:384
: > gpurun_out/g44_time.txt
for rep in 1 2; do
  for v in cur pw2; do
    timeout -k 10 120 python tools/time_variant.py $L/libsrsran_ldpc_hip_$v.so sweep $SW >> gpurun_out/g44_time.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/g44_time.txt
