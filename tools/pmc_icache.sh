cd /root/repo && mkdir -p gpurun_out/pmcic && export TMPDIR=/tmp
timeout -k 10 200 python tools/time_et.py > gpurun_out/et.txt 2>&1; grep -v amdgpu.ids gpurun_out/et.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmcic -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-baseline off --extras off > gpurun_out/pmcic/log.txt 2>&1
echo pmc rc=$?
