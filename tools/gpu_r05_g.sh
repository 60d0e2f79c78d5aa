#!/bin/bash
# Round 5, GPU call G: where a one-CB call's time goes on the work-queue path with the lane-split decoder
# (tools/diag_dwq.py on diagnostic builds: make VARIANT=diagdwq FLAGS="-DLDPC_HIP_DIAG_DWQ -DLDPC_HIP_DIAG_CB";
# diagdwq0 = the same build of the previous sources), alternating, two rounds.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
: > gpurun_out/diag_dwq_r05.txt
for r in 1; do
  for v in diagdwq; do
    echo "== $v" >> gpurun_out/diag_dwq_r05.txt
    DIAG_LIB=$v timeout -k 10 300 python3 -u tools/diag_dwq.py 200 >> gpurun_out/diag_dwq_r05.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/diag_dwq_r05.txt
