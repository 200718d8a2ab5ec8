#!/bin/bash
# Round 3 session F: K = 4 sweeps in 2-row waves (natural rows, no unroll) against the K = 3 default.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --steps 48 --warmup 12"
scripts/gpu_session.sh "wtk=$PYT tests/test_gpu_temporal.py -k 'wtk'" \
  "k3=$B" "k4r2w8=MDFX_WTK_K4RY=2 MDFX_WTK_WB=8 $B --temporal 4" "k4r2w4=MDFX_WTK_K4RY=2 MDFX_WTK_WB=4 $B --temporal 4" \
  "k4r1=$B --temporal 4" "k3_b=$B" "k4r2w8_b=MDFX_WTK_K4RY=2 MDFX_WTK_WB=8 $B --temporal 4" \
  "k4r2w8_drv=MDFX_WTK_K4RY=2 MDFX_WTK_WB=8 python bench.py --steps 20 --warmup 5 --temporal 4" || exit $?
PMC_TAG=k4r2 MDFX_WTK_K4RY=2 MDFX_WTK_WB=8 BENCH_ARGS="--temporal 4" scripts/gpu_session.sh pmc_fetch || exit $?
for f in k3 k4r2w8 k4r2w4 k4r1 k3_b k4r2w8_b k4r2w8_drv; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
