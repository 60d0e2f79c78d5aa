# GPU box: the whole -m gpu suite, then bench.py's HAL extra alone (C4 slot through the plugins, p50 of 20).
cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "
import json, torch, bench
from srsran_projectvtlmo_amd import _lib
ctx = _lib.Context(0); s = torch.cuda.Stream()
for rep in range(2):
    r = bench.extra_hal(ctx, s)
    print(json.dumps({k: r['pusch_dec'][k] for k in ('slot_us_p50', 'slot_us_p99', 'tb0_us_p50', 'cbs_crc_ok')}))
ctx.close()" > gpurun_out/hal.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/hal.txt; exit $rc
