# GPU box: N=2 rehearsal of bench.py on one GPU (two ranks share it) and a kernel trace of one replayed C4 slot
cd /root/repo && mkdir -p gpurun_out/pc4 && export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_n2.log 2>&1
rc=$?; echo "n2 rc=$rc"; tail -c 700 gpurun_out/bench_n2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc4 -o run -- python3 tools/c4_trace.py > gpurun_out/pc4/c4.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
