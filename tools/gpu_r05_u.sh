#!/bin/bash
# Round 5, GPU call U: the encoder kernel's own time on device-resident messages (tools/time_encoder.py), and a kernel
# trace of the same.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/time_encoder.py > gpurun_out/time_encoder_r05u.txt 2>&1
rc=$?; cat gpurun_out/time_encoder_r05u.txt | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enc_r05u -o run -- python3 tools/time_encoder.py > gpurun_out/prof_enc_r05u.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
