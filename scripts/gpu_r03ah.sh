#!/bin/bash
# Round 3 session AH: the K = 2 cliff on the thin N = 8 slab (461 GCells/s per GPU, below a single sweep?): K = 1 proxy and a kernel trace of the K = 2 proxy.
set -o pipefail
cd "$(dirname "$0")/.."
P="python bench.py --steps 48 --warmup 12 --rank-proxy 8"
scripts/gpu_session.sh "k1=$P --temporal 1" "k2v=$P --temporal 2 --graph off" || exit $?
PROF_TAG=ah_k2 BENCH_ARGS="--steps 48 --warmup 12 --rank-proxy 8 --temporal 2 --graph off" scripts/gpu_session.sh prof || exit $?
for f in k1 k2v; do echo "$f $(grep -o '"value": [0-9.]*\|"temporal_block": [0-9]*' gpurun_out/$f.log | tr '\n' ' ')"; done
