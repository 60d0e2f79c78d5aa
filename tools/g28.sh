# GPU box: per-step spans of the pipelined specialised decoder (diag build) and the default bench line
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python tools/diag_spec.py 8 diag > gpurun_out/g28_steps.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/g28_bench.log 2>&1
rc=$?; tail -c 3000 gpurun_out/g28_bench.log; exit $rc
