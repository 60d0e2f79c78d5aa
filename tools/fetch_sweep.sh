#!/bin/bash
# GPU box: raw FETCH_SIZE / WRITE_SIZE of the C2 decoder (BG1 Z=384, 8 it) against the codeblocks per launch, for the
# product library and the variant without the split-row address table (LDPC_SPEC_SPLIT_LDS_ROWS=0: the split rows'
# addresses computed in the step, no table copy in the prologue), one --pmc pass per counter, size and library
# (tools/time_variant.py launches the batch 12 times). tools/fetch_fit.py then fits raw = a*N + b per library.
#   fetch_sweep.sh [variant...]     (default: notab; "cur" = the product library, always run)
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
L=srsran_projectvtlmo_amd/lib
VARS=("cur" "${@:-notab}")
for v in "${VARS[@]}"; do
  case $v in cur) f=$L/libsrsran_ldpc_hip.so ;; *) f=$L/libsrsran_ldpc_hip_$v.so ;; esac
  mkdir -p gpurun_out/fetch/$v
  for n in 8 64 128 256; do
    for c in FETCH_SIZE WRITE_SIZE; do
      [ "$v" != cur ] && [ "$c" = WRITE_SIZE ] && continue
      d=gpurun_out/fetch/$v/${c}_$n
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- \
        python3 tools/time_variant.py "$f" 1 384 8 $n > $d.log 2>&1
      rc=$?; echo "$v $c N=$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
    done
  done
done
exit 0
