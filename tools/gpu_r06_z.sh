#!/bin/bash
# GPU box (round 6): four lanes per check node for the Z = 36 / 40 one-wave graphs (LDPC_SPEC_QUAD_P4_MAX_Z=40,
# libsrsran_ldpc_hip_p4z40.so) against the product (copied to _base.so): smoke() bit-exactness and 128-CB batch times
# per library (tools/batch_time_lib.py, alternating), then the host-memory routes A/B (tools/route_ab.py).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for lib in base p4z40; do
    timeout -k 10 300 python3 -u tools/batch_time_lib.py $lib 20 >> gpurun_out/r06z_batch.txt 2>> gpurun_out/r06z_batch.err || exit 1
  done
done
cat gpurun_out/r06z_batch.txt
timeout -k 10 500 python3 -u tools/route_ab.py 3 base:LIB=base p4z40:LIB=p4z40 > gpurun_out/r06z_route_ab.json 2> gpurun_out/r06z_route_ab.err
rc=$?; tail -c 300 gpurun_out/r06z_route_ab.err; exit $rc
