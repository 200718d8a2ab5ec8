#!/bin/bash
# Round 4 session C, in three gpurun calls (each under gpurun's 1200 s limit):
#   part 1: the GPU test tier (pencil tests first, then the rest)
#   part 2: the round-3 tree (ab_alt/, commit 791b0ce) against this tree on one box, interleaved
#           (headline bench, N = 8 / 4 slab proxies), the pencil proxies, the heat7_wxk diagnostics
#   part 3: graph replay vs eager under HIP runtime settings (bench/graph_probe.py); graph vs eager
#           kernel traces of the N = 8 proxy
#   part 4: the driver's N = 8 path rehearsed with 8 processes sharing the GPU (full gate / trial flow)
set -o pipefail
cd "$(dirname "$0")/.."
part=${1:-1}
B="--steps 20 --warmup 5"
P8="--rank-proxy 8 --steps 48 --warmup 5"
P4="--rank-proxy 4 --steps 48 --warmup 5"
if [[ $part == 1 ]]; then
  LIMIT=360 scripts/gpu_session.sh "pencil=python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu -k pencil tests/test_gpu_engine.py tests/test_gpu_proxy.py tests/test_gpu_ipc.py" || exit $?
  LIMIT=780 scripts/gpu_session.sh "gputests=python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -k 'not pencil' tests" || exit $?
  grep -E "passed|failed" gpurun_out/pencil.log gpurun_out/gputests.log | tail -4
  N1="--graph off --steps 50 --warmup 10"
  Q4="--rank-proxy 4 --graph off --rounds 1 --steps 48 --warmup 5"
  scripts/gpu_session.sh "n3_a=python ab_alt/bench.py $N1" "n4_a=python bench.py $N1" "n3_b=python ab_alt/bench.py $N1" "n4_b=python bench.py $N1" \
    "q3=python ab_alt/bench.py $Q4" "q4=python bench.py $Q4" "q3b=python ab_alt/bench.py $Q4" "q4b=python bench.py $Q4" \
    "b4=python bench.py $B" "p8=python bench.py $P8" "p8pen=python bench.py $P8 --py 2" "p4=python bench.py $P4" || exit $?
  for f in n3_a n4_a n3_b n4_b q3 q4 q3b q4b b4 p8 p8pen p4; do
    echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
elif [[ $part == 2 ]]; then
  scripts/gpu_session.sh "r4_p8pen=python bench.py $P8 --py 2" "r4_p8pen4=python bench.py $P8 --py 4" "r4_p4pen=python bench.py $P4 --py 2" \
    "r3_a=python ab_alt/bench.py $B" "r4_a=python bench.py $B" "r3_b=python ab_alt/bench.py $B" "r4_b=python bench.py $B" \
    "r3_p8a=python ab_alt/bench.py $P8" "r4_p8a=python bench.py $P8" "r3_p8b=python ab_alt/bench.py $P8" "r4_p8b=python bench.py $P8" \
    "r3_p4=python ab_alt/bench.py $P4" "r4_p4=python bench.py $P4" || exit $?
  scripts/gpu_session.sh "diag=python bench/kernel_ab.py --n 1024 --iters 10 --rounds 3 --variants 'STEPS=4;STEPS=4,DIAG=1;STEPS=4,DIAG=2;STEPS=4,DIAG=3;STEPS=4,DIAG=4;STEPS=4,DIAG=5;STEPS=4,DIAG=7'" || exit $?
  for f in r3_a r4_a r3_b r4_b r3_p8a r4_p8a r3_p8b r4_p8b r3_p4 r4_p4 r4_p8pen r4_p8pen4 r4_p4pen; do
    echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
elif [[ $part == 3 ]]; then
  # no-trial A/B (round-3 tree vs this one): kernel traces of the N = 1 headline, the N = 4 proxy
  # (overlap trial only) and its exchange variants (mailbox protocol, serial pulls)
  N1="--graph off --steps 50 --warmup 10"
  Q4="--rank-proxy 4 --graph off --rounds 1 --steps 48 --warmup 5"
  PR="cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv"
  scripts/gpu_session.sh "t3=$PR -d $PWD/gpurun_out/t3 -o run -- python3 $PWD/ab_alt/bench.py $N1" \
    "t4=$PR -d $PWD/gpurun_out/t4 -o run -- python3 $PWD/bench.py $N1" \
    "q3=python ab_alt/bench.py $Q4" "q4=python bench.py $Q4" "q4_mbox=MDFX_IPC_DIRECT=0 python bench.py $Q4" \
    "q4_ser=MDFX_XPULL=serial python bench.py $Q4" "q4_mser=MDFX_IPC_DIRECT=0 MDFX_XPULL=serial python bench.py $Q4" \
    "q3b=python ab_alt/bench.py $Q4" "q4b=python bench.py $Q4" || exit $?
  for f in t3 t4 q3 q4 q4_mbox q4_ser q4_mser q3b q4b; do
    echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
  LIMIT=600 scripts/gpu_session.sh "gprobe2=python bench/graph_probe.py --temporal 2" "gprobe4=python bench/graph_probe.py --temporal 4 --rounds 1" || exit $?
  PROF_TAG=p8g1 BENCH_ARGS="--rank-proxy 8 --steps 24 --warmup 4 --graph on --rounds 1 --overlap" scripts/gpu_session.sh prof || exit $?
  PROF_TAG=p8e1 BENCH_ARGS="--rank-proxy 8 --steps 24 --warmup 4 --graph off --rounds 1 --overlap" scripts/gpu_session.sh prof || exit $?
elif [[ $part == 4 ]]; then
  LIMIT=300 scripts/gpu_session.sh "churn_nobar=MDFX_IPC_CLOSE_BARRIER=0 python scripts/ipc_churn.py --world 8" \
    "churn=python scripts/ipc_churn.py --world 8" || exit $?
  tail -3 gpurun_out/churn_nobar.log gpurun_out/churn.log
  LIMIT=1000 scripts/gpu_session.sh "share8=python bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 --verbose" || exit $?
  echo "share8 $(grep -o '"value": [0-9.]*' gpurun_out/share8.log) $(grep -o '"parallelism": "[^"]*"' gpurun_out/share8.log)"
fi
