#!/bin/bash
# Round 3 session I: heat7_wxk edge waves with fewer own rows (balanced plane work), K = 4.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --steps 48 --warmup 12"
scripts/gpu_session.sh "wxk=$PYT tests/test_gpu_temporal.py -k 'wxk'" || exit $?
grep -q ' passed' gpurun_out/wxk.log && ! grep -q 'failed' gpurun_out/wxk.log || { tail -30 gpurun_out/wxk.log; exit 1; }
scripts/gpu_session.sh "r31=$B" "r22=MDFX_WXK_RY=2 $B" "r21=MDFX_WXK_RY=21 $B" "r31_b=$B" "r22_b=MDFX_WXK_RY=2 $B" "r21_b=MDFX_WXK_RY=21 $B" \
  "drv=python bench.py --steps 20 --warmup 5" "p8=python bench.py --rank-proxy 8 --steps 48 --warmup 12" \
  "p8r22=MDFX_WXK_RY=2 python bench.py --rank-proxy 8 --steps 48 --warmup 12" "n512=$B --n 512" "n512r22=MDFX_WXK_RY=2 $B --n 512" || exit $?
PMC_TAG=r31 scripts/gpu_session.sh pmc_fetch || exit $?
for f in r31 r22 r21 r31_b r22_b r21_b drv p8 p8r22 n512 n512r22; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
