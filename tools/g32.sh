# GPU box: mid-size specialised graphs (mid) vs the product library: C3, then 128-CB batches of the added graphs
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
SW=1:240,1:208,1:160,1:128,2:240,2:208,2:160,2:128
for rep in 1 2; do
  for v in "" mid; do
    f=$L/libsrsran_ldpc_hip${v:+_$v}.so
    timeout -k 10 180 python tools/time_c3.py $f >> gpurun_out/g32_time.txt 2>&1 || exit 1
    timeout -k 10 180 python tools/time_variant.py $f sweep $SW >> gpurun_out/g32_time.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/g32_time.txt
