#!/bin/bash
# Round 5, GPU call T: the N = 2 path of bench.py rehearsed on a one-GPU box (two ranks share GPU 0; gloo barrier and
# max-over-ranks timing; each rank's extra is its own C4 cell, C5), at HEAD.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_n2_r05.log 2>&1
rc=$?; echo "n2 rc=$rc"; grep '^{' gpurun_out/bench_n2_r05.log | tail -1 | cut -c1-600; exit $rc
