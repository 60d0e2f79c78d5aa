#!/bin/bash
# Round 5, GPU call R: extra.hal with the copy work queue off / on, both with LDPC_HIP_DWQ_IDLE_US=20000 (resident
# grids stay between the bench's slots, as in continuous slot-by-slot operation), alternating, two rounds.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 1; do
    LDPC_HIP_DWQ_IDLE_US=20000 LDPC_HIP_HAL_DWQ_COPY=$v timeout -k 10 300 python3 -u tools/run_hal_bench.py 20 > gpurun_out/hal_r05r_c${v}_$r.json 2> gpurun_out/hal_r05r_c${v}_$r.log
    rc=$?; echo "copy=$v round $r rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 -c "import json,sys; d=json.load(open('gpurun_out/hal_r05r_c${v}_$r.json')); print(d['pusch_dec']['slot_us_p50'], d['pusch_dec_phases_us_p50']['multi_cb_tb'], {k: v['slot_us_p50'] for k, v in d['pusch_dec_concurrent'].items()}, d['pdsch_enc']['tb_mode_slot_us_p50'])"
  done
done
exit 0
