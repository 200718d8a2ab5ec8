#!/bin/bash
# Round 3 session M: full GPU tier with the cost-model band choice and the 27-point K = 3 default
# (fp64, rows >= 1024), then the configs, then why the fp64 heat7_wxk sweep is slow (SQ counters).
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=1100 scripts/gpu_session.sh gputests smoke || exit $?
B="python bench.py --steps 48 --warmup 12"
P="python bench.py --steps 48 --warmup 12 --rank-proxy"
scripts/gpu_session.sh "h1=$B" "hdrv=python bench.py --steps 20 --warmup 5" "h2=$B" "p8=$P 8" "p4=$P 4" "p2=$P 2" "h512=$B --n 512" \
  "b27f32=$B --stencil box27 --n 512" "b27f64=$B --stencil box27 --n 512 --dtype f64" "b27f32_1024=python bench.py --stencil box27 --n 1024 --steps 24 --warmup 6" \
  "f64r=python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12" || exit $?
TAG=f64wtk BENCH_ARGS="--dtype f64" bash scripts/pmc_sq.sh || exit $?
TAG=f64wxk MDFX_H7_WXK=1 BENCH_ARGS="--dtype f64" bash scripts/pmc_sq.sh || exit $?
for f in h1 hdrv h2 p8 p4 p2 h512 b27f32 b27f64 b27f32_1024 f64r; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep -E 'passed|failed' gpurun_out/gputests.log | tail -1
