#!/bin/bash
# heat7_wtk fp32 8-wave bands: two vs three window buffers (MDFX_WTK_NBUF), tests first.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh \
  "nb_tests=MDFX_WTK_NBUF=3 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -k wtk" \
  "nb_2a=$B" "nb_3a=MDFX_WTK_NBUF=3 $B" "nb_2b=$B" "nb_3b=MDFX_WTK_NBUF=3 $B" \
  "nb_2048_2=$B --n 2048 --steps 24 --warmup 6" "nb_2048_3=MDFX_WTK_NBUF=3 $B --n 2048 --steps 24 --warmup 6" || exit $?
for f in gpurun_out/nb_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
