cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/run_variants.sh _pair _pairns _old
