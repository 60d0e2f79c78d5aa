cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pc4n -o run -- python3 tools/c4_trace.py llrs nomixed > gpurun_out/pc4n.log 2>&1 || exit 1
python3 tools/trace_timeline.py gpurun_out/pc4n 16
