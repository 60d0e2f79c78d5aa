# Decoder edge-split threshold sweep on the C2 bench (diagnostic).
for v in 99 11 8 6 3; do
  echo "== SPLIT_MINDEG=$v"
  LDPC_HIP_SPLIT_MINDEG=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-baseline off 2>&1 | grep -o '"kernel_ms_per_step": [0-9.]*' || exit 1
done
