#!/bin/bash
# GPU box: one PMC pass per variant library over tools/time_variant.py (C2 batch). Usage: pmc_variants.sh suffix...
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcv
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
C2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"
for v in "$@"; do
  for i in 1 2; do
    eval C=\$C$i
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmcv/$v$i -o run -- python3 tools/time_variant.py srsran_projectvtlmo_amd/lib/libsrsran_ldpc_hip$v.so > gpurun_out/pmcv/$v$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
