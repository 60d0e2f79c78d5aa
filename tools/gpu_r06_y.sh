#!/bin/bash
# GPU box (round 6): the host-memory routes with fewer work-queue hardware queues than keys in use
# (LDPC_HIP_DWQ_MAX_QUEUES 3 / 2 / 1): what a decode key pays when a PDSCH encoder or copy grid holds a queue and the
# key is refused (the launch path serves it). tools/route_ab.py, two alternating rounds.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/route_ab.py 2 q3:LDPC_HIP_DWQ_MAX_QUEUES=3 q2:LDPC_HIP_DWQ_MAX_QUEUES=2 q1:LDPC_HIP_DWQ_MAX_QUEUES=1 > gpurun_out/r06y_queue_cap.json 2> gpurun_out/r06y_queue_cap.err
rc=$?; tail -c 400 gpurun_out/r06y_queue_cap.err; exit $rc
