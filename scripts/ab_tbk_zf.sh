#!/bin/bash
# heat7_tbk with the z-held factor: bitwise tests, then the K = 2 shapes.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh \
  "zf_tests=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py" \
  "zf_512=$B --n 512" "zf_1024_k2=$B --temporal 2" "zf_1024f64_k2=$B --dtype f64 --temporal 2" "zf_512b=$B --n 512" || exit $?
for f in gpurun_out/zf_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
