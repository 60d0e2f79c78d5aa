# GPU box: A/B of the early role's late addresses (late) and the SGPR packed one (product) vs the committed kernel (pipe)
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
SW=1:384,1:352,1:320,1:288,1:256,2:384,2:352,2:320,2:288,2:256
for rep in 1 2; do
  for v in pipe late ""; do
    f=$L/libsrsran_ldpc_hip${v:+_$v}.so
    timeout -k 10 120 python tools/time_variant.py $f sweep $SW >> gpurun_out/g31_time.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/g31_time.txt
