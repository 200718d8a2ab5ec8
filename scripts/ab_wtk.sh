#!/bin/bash
# heat7_wtk: bitwise tests, then the default dispatch at 1024^3 fp32 / fp64, 2048^3 fp64 + residual
# and the 8-slab shape.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh \
  "wtk_tests=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -k wtk" \
  "ab_n1_a=$B" "ab_v8=$B --virtual-ranks 8" "ab_f64=$B --dtype f64" "ab_n1_b=$B" \
  "ab_2048f64_res=python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12" || exit $?
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*\|"temporal_block": [0-9]*' $f | tr '\n' ' ')"; done
