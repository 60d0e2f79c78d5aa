# GPU box: small-Z specialised kernels (experiment build "small"): parity of the specialised-graph cases, then timing
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
V=srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip_small.so
P=srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip.so
timeout -k 10 200 python tools/check_spec_graphs.py $V 2:36,1:36,2:5,1:2 > gpurun_out/g34.txt 2>&1 || { cat gpurun_out/g34.txt | tail -30; exit 1; }
for f in $P $V $P $V; do
  timeout -k 10 120 python tools/time_variant.py $f sweep 2:36,1:36,2:5,1:2 >> gpurun_out/g34.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/g34.txt
