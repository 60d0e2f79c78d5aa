cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/run_variants.sh "" && \
timeout -k 10 120 python tools/diag_spec.py 8 diag > gpurun_out/diag_light.txt 2>&1 && \
timeout -k 10 120 python tools/diag_spec.py 8 diagfull > gpurun_out/diag_full.txt 2>&1
echo rc=$?; head -3 gpurun_out/diag_light.txt; tail -2 gpurun_out/diag_light.txt; head -3 gpurun_out/diag_full.txt
