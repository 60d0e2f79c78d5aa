cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_quick.txt 2>&1
echo "bench rc=$?"; tail -c 1500 gpurun_out/bench_quick.txt
