cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 tools/ubench/valu4 > gpurun_out/valu4.txt 2>&1 &&
timeout -k 10 60 tools/ubench/valu2 > gpurun_out/valu2.txt 2>&1 &&
timeout -k 10 60 tools/ubench/valu3 > gpurun_out/valu3.txt 2>&1 &&
timeout -k 10 180 python tools/diag_steps.py diag > gpurun_out/diag.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off --extras off > gpurun_out/bench0.txt 2>&1
