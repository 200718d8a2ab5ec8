#!/bin/bash
set -o pipefail
cd /root/repo
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh "ab_v8_k2=$B --virtual-ranks 8 --temporal 2" "ab_b27_v8=$B --stencil box27 --n 512 --virtual-ranks 8" \
  "ab_b27f64_v4=$B --stencil box27 --dtype f64 --n 512 --virtual-ranks 4" "ab_v8_k3=$B --virtual-ranks 8" "ab_n1=$B" \
  "tests_tmp=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_engine.py" || exit $?
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
