cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
G=1:256,1:288,1:320,2:256,2:288,2:320,2:352,2:384,1:384
for v in "" _s8 _s6 _s4; do
  timeout -k 10 200 python tools/time_variant.py srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip$v.so sweep $G || exit 1
done
