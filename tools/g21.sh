cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python tools/diag_phase.py 2 36 > gpurun_out/phase_bg2_z36.txt 2>&1 && \
timeout -k 10 120 python tools/diag_phase.py 1 128 > gpurun_out/phase_bg1_z128.txt 2>&1
rc=$?; head -40 gpurun_out/phase_bg2_z36.txt; exit $rc
