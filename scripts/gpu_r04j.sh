#!/bin/bash
# Round 4 session J: 2-wave heat7_wxk bands for the pencil y strips (MDFX_WXK_STRIP=0: the 8-wave
# bands): pencil GPU tests, then the N = 8 4 x 2 / 2 x 4 pencil proxies A/B and a trace.
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=400 scripts/gpu_session.sh "t_pen=python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k pencil tests" || exit $?
grep -E "passed|failed" gpurun_out/t_pen.log | tail -1
grep -q " failed" gpurun_out/t_pen.log && exit 1
Q="--steps 48 --warmup 5 --graph off --rounds 1 --overlap"
scripts/gpu_session.sh "s8=python bench.py --rank-proxy 8 --py 2 $Q" "o8=MDFX_WXK_STRIP=0 python bench.py --rank-proxy 8 --py 2 $Q" \
  "s8b=python bench.py --rank-proxy 8 --py 2 $Q" "o8b=MDFX_WXK_STRIP=0 python bench.py --rank-proxy 8 --py 2 $Q" \
  "s84=python bench.py --rank-proxy 8 --py 4 $Q" "o84=MDFX_WXK_STRIP=0 python bench.py --rank-proxy 8 --py 4 $Q" \
  "s8t=python bench.py --rank-proxy 8 --py 2 --steps 48 --warmup 5" "slab8t=python bench.py --rank-proxy 8 --steps 48 --warmup 5" || exit $?
A="--rank-proxy 8 --py 2 --steps 24 --warmup 4 --graph off --rounds 1 --overlap"
PROF_TAG=pen8 BENCH_ARGS="$A" scripts/gpu_session.sh prof || exit $?
for f in s8 o8 s8b o8b s84 o84 s8t slab8t; do
  echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
