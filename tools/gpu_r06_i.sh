#!/bin/bash
# Round 6, call I: the N>1 bench path rehearsed on one GPU: without --allow-shared-device it must refuse (two ranks
# on one GPU); with it, the line carries config.devices and devices_distinct=false, and C5 runs one cell per rank
set -o pipefail
mkdir -p gpurun_out
P=$((29500 + RANDOM % 1000))
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --steps 20 --warmup 5 --extras off > gpurun_out/r06i_refuse.log 2>&1
echo "refuse rc=$?" >> gpurun_out/r06i_refuse.log
P=$((P + 1))
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --steps 20 --warmup 5 --allow-shared-device > gpurun_out/r06i_rehearsal.log 2>&1
