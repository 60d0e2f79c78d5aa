# GPU box: A/B of precomputed split-row addresses (sa1: row 0, sa2: rows 0-1) against none (sa0), BG1 graphs (the only
# ones with split rows) at 128 CBs, 8 it; two rounds.
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
SW=1:384,1:320,1:256,1:208,1:128,1:64
: > gpurun_out/g43_time.txt
for rep in 1 2; do
  for v in sa0 sa1 sa2; do
    timeout -k 10 120 python tools/time_variant.py $L/libsrsran_ldpc_hip_$v.so sweep $SW >> gpurun_out/g43_time.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/g43_time.txt
