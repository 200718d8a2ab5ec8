#!/bin/bash
# heat7_wtk fp64 rows per wave in 8-wave bands: tests, then the default dispatch.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh \
  "ry_tests=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -k wtk" \
  "ry_f64=$B --dtype f64" "ry_2048f64=$B --n 2048 --dtype f64 --steps 24 --warmup 6" \
  "ry_2048f64_res=python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12" "ry_f32=$B" || exit $?
for f in gpurun_out/ry_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
