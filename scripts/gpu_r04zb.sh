#!/bin/bash
# Round 4, session Z (part 2): the c5 configs with the warm-up aligned to the residual interval.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/zb
v() { grep -o '"value": [0-9.]*' "$1" | head -1; }
timeout -k 10 300 python bench.py --n 2048 --dtype f64 --steps 24 --warmup 12 --residual-every 12 > gpurun_out/zb/c5_r12.json 2>/dev/null || exit 1
echo "c5 every 12 $(v gpurun_out/zb/c5_r12.json)"
timeout -k 10 300 python bench.py --n 2048 --dtype f64 --steps 20 --warmup 10 --residual-every 10 > gpurun_out/zb/c5_r10.json 2>/dev/null || exit 1
echo "c5 every 10 $(v gpurun_out/zb/c5_r10.json)"
timeout -k 10 300 python bench.py --rank-proxy 8 --n 2048 --dtype f64 --steps 24 --warmup 12 --residual-every 12 > gpurun_out/zb/c5_p8.json 2>/dev/null || exit 1
echo "c5 proxy8 $(v gpurun_out/zb/c5_p8.json)"
