for v in 99 19 8 3; do
  echo "== SPLIT_MINDEG=$v"
  LDPC_HIP_SPLIT_MINDEG=$v timeout -k 10 120 python tools/diag_steps.py diag 2>&1 | head -3
done
