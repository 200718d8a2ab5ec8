#!/bin/bash
# heat7 wide-row (x-tiled heat7_tb2) check after a kernel change: bitwise tests, then the fp64
# BASELINE config and the wide fp32 / fp64 cubes.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -k "xtiled or fused_two_steps or stale or wide" -x 2>&1 | tail -1 || exit 1
b() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['ms_per_step'], d.get('pct_of_hbm_copy_roof'))"; }
echo "== 2048^3 f64 + residual"; b --dtype f64 --n 2048 --residual-every 10 --steps 20 --warmup 4 || exit 1
echo "== 1024^3 f64"; b --dtype f64 --n 1024 --steps 30 --warmup 6 || exit 1
echo "== 2048^3 f32"; b --n 2048 --steps 20 --warmup 4 || exit 1
