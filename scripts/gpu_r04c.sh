#!/bin/bash
# Round 4 session C: the whole GPU test tier on the pruned tree; the round-3 tree (ab_alt/, commit 791b0ce) against this tree on one box
# (headline bench and N = 8 / 4 proxies, interleaved); the graph-replay regression test; the
# driver's N = 8 path rehearsed with 8 processes sharing the GPU (full gate / trial flow).
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
LIMIT=700 scripts/gpu_session.sh "gputests=python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" || exit $?
grep -q " passed" gpurun_out/gputests.log && ! grep -q "failed" gpurun_out/gputests.log || { tail -40 gpurun_out/gputests.log; exit 1; }
B="--steps 20 --warmup 5"
P8="--rank-proxy 8 --steps 48 --warmup 5"
P4="--rank-proxy 4 --steps 48 --warmup 5"
scripts/gpu_session.sh "r3_a=python ab_alt/bench.py $B" "r4_a=python bench.py $B" "r3_b=python ab_alt/bench.py $B" "r4_b=python bench.py $B" \
  "r3_c=python ab_alt/bench.py $B" "r4_c=python bench.py $B" \
  "r3_p8a=python ab_alt/bench.py $P8" "r4_p8a=python bench.py $P8" "r3_p8b=python ab_alt/bench.py $P8" "r4_p8b=python bench.py $P8" \
  "r3_p4=python ab_alt/bench.py $P4" "r4_p4=python bench.py $P4" || exit $?
scripts/gpu_session.sh "diag=python bench/kernel_ab.py --n 1024 --iters 10 --rounds 3 --variants 'STEPS=4;STEPS=4,DIAG=1;STEPS=4,DIAG=2;STEPS=4,DIAG=3;STEPS=4,DIAG=4;STEPS=4,DIAG=5;STEPS=4,DIAG=7'" || exit $?
PROF_TAG=p8g1 BENCH_ARGS="--rank-proxy 8 --steps 24 --warmup 4 --graph on --rounds 1 --overlap" scripts/gpu_session.sh prof || exit $?
PROF_TAG=p8e1 BENCH_ARGS="--rank-proxy 8 --steps 24 --warmup 4 --graph off --rounds 1 --overlap" scripts/gpu_session.sh prof || exit $?
LIMIT=900 scripts/gpu_session.sh "share8=python bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 --verbose" || exit $?
for f in r3_a r4_a r3_b r4_b r3_c r4_c r3_p8a r4_p8a r3_p8b r4_p8b r3_p4 r4_p4 share8; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"transport": "[a-z_]*"' gpurun_out/$f.log | head -1)"; done
