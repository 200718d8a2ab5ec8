#!/bin/bash
# Round 3 session J: heat7_wxk 5-step sweeps (2-row inner / 1-row edge waves, 160 KB LDS).
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "wxk=$PYT tests/test_gpu_temporal.py -k 'wxk'" || exit $?
grep -q ' passed' gpurun_out/wxk.log && ! grep -q 'failed' gpurun_out/wxk.log || { tail -30 gpurun_out/wxk.log; exit 1; }
B="python bench.py --steps 60 --warmup 20"
scripts/gpu_session.sh "k4=$B" "k5=$B --temporal 5" "k4_b=$B" "k5_b=$B --temporal 5" \
  "k5drv=python bench.py --steps 20 --warmup 5 --temporal 5" "k4drv=python bench.py --steps 20 --warmup 5" \
  "n512k4=$B --n 512" "n512k5=$B --n 512 --temporal 5" "n3072k5=python bench.py --n 3072 --steps 10 --warmup 5 --temporal 5" \
  "p8k5=python bench.py --rank-proxy 8 --steps 60 --warmup 20 --temporal 5" || exit $?
PMC_TAG=k5 BENCH_ARGS="--temporal 5" scripts/gpu_session.sh pmc_fetch || exit $?
for f in k4 k5 k4_b k5_b k5drv k4drv n512k4 n512k5 n3072k5 p8k5; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
