#!/bin/bash
# Round 6, call H: (1) the address-arithmetic bound of C2: timing-only variants without the wrap (nowrap) and without
# any per-position address op (noaddr) against the product, alternating 3 rounds; (2) the bench with the pool at 3
# queues (HAL and software-route extras)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 bash tools/ab_variants.sh r06h_addr_ab 3 1:384,2:384,1:256,2:208 cur nowrap noaddr > /dev/null 2>&1 &&
timeout -k 10 400 python3 -u bench.py --extras-out gpurun_out/r06h_extras.json > gpurun_out/r06h_bench.log 2> gpurun_out/r06h_bench.err
