#!/bin/bash
# heat7_wtk fp64 rows per wave (2 vs 3) and fp64 2048^3 K = 3 vs K = 2; fp32 RY 2 vs 3.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh \
  "ab_f64_k3_r3=$B --dtype f64 --temporal 3" "ab_f64_k3_r2=MDFX_WTK_RY=2 $B --dtype f64 --temporal 3" \
  "ab_f64_k2=$B --dtype f64 --temporal 2" \
  "ab_f32_r2=MDFX_WTK_RY=2 $B --temporal 3" "ab_f32_r3=$B --temporal 3" \
  "ab_f64_k3_r3b=$B --dtype f64 --temporal 3" "ab_f64_k3_r2b=MDFX_WTK_RY=2 $B --dtype f64 --temporal 3" \
  "ab_2048f64_k2=$B --n 2048 --dtype f64 --steps 24 --warmup 6 --temporal 2" \
  "ab_2048f64_k3=$B --n 2048 --dtype f64 --steps 24 --warmup 6 --temporal 3" \
  "ab_2048f64_k3r2=MDFX_WTK_RY=2 $B --n 2048 --dtype f64 --steps 24 --warmup 6 --temporal 3" \
  "ab_2048f32_k2=$B --n 2048 --steps 24 --warmup 6 --temporal 2" \
  "ab_2048f32_k3=$B --n 2048 --steps 24 --warmup 6 --temporal 3" || exit $?
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*\|"temporal_block": [0-9]*' $f | tr '\n' ' ')"; done
