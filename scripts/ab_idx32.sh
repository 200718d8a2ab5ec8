#!/bin/bash
# 32-bit row / plane indices in heat7_tbk and box27_tbk: bitwise tests, then the K = 2 shapes.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh \
  "idx_tests=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_kernels.py" \
  "i_512=$B --n 512" "i_1024_k2=$B --temporal 2" "i_b27f64=$B --stencil box27 --dtype f64 --n 512" \
  "i_b27f32=$B --stencil box27 --n 512" "i_1024f64_k2=$B --dtype f64 --temporal 2" || exit $?
for f in gpurun_out/i_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
