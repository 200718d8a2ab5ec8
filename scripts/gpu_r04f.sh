#!/bin/bash
# Round 4 session F: kernel traces of the N = 8 rank proxy - slab (blit / SDMA face copies) and 4 x 2
# pencil - at the configuration the bench picks (eager, one round, overlapped).
set -o pipefail
cd "$(dirname "$0")/.."
A="--rank-proxy 8 --steps 24 --warmup 4 --graph off --rounds 1 --overlap"
PROF_TAG=p8 BENCH_ARGS="$A" scripts/gpu_session.sh prof || exit $?
PROF_TAG=p8sdma BENCH_ARGS="$A --transport proxy_sdma" scripts/gpu_session.sh prof || exit $?
PROF_TAG=p8pen BENCH_ARGS="$A --py 2" scripts/gpu_session.sh prof || exit $?
for t in p8 p8sdma p8pen; do
  echo "== $t $(grep -o '"value": [0-9.]*' gpurun_out/prof_$t.log)"
  python3 scripts/kernel_timeline.py gpurun_out/prof_$t --skip 40 | head -40
done
