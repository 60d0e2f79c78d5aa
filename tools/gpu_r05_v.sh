#!/bin/bash
# Round 5, GPU call V: the work queue's runtime knobs against the HAL C4 slot (extra.hal), two alternating rounds:
# default, LDPC_HIP_DWQ_WORKGROUPS=8 / 64, LDPC_HIP_DWQ_SPREAD=0, LDPC_HIP_DWQ_IDLE_US=20000.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "default" "LDPC_HIP_DWQ_WORKGROUPS=8" "LDPC_HIP_DWQ_WORKGROUPS=64" "LDPC_HIP_DWQ_SPREAD=0" "LDPC_HIP_DWQ_IDLE_US=20000"; do
    tag=$(echo "$cfg" | tr '=' '_')
    if [ "$cfg" = "default" ]; then
      timeout -k 10 300 python3 -u tools/run_hal_bench.py 20 > gpurun_out/hal_r05v_${tag}_$r.json 2> /dev/null
    else
      env "$cfg" timeout -k 10 300 python3 -u tools/run_hal_bench.py 20 > gpurun_out/hal_r05v_${tag}_$r.json 2> /dev/null
    fi
    rc=$?; [ $rc -ne 0 ] && { echo "$cfg rc=$rc"; exit $rc; }
    python3 -c "import json; d=json.load(open('gpurun_out/hal_r05v_${tag}_$r.json')); print('$cfg', $r, d['pusch_dec']['slot_us_p50'], d['pusch_dec_phases_us_p50']['one_cb_tb'], {k: v['slot_us_p50'] for k, v in d['pusch_dec_concurrent'].items()}, d['pdsch_enc']['tb_mode_slot_us_p50'])"
  done
done
exit 0
