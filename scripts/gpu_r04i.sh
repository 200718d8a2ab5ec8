#!/bin/bash
# Round 4 session I: the folded lower boundary (interior sweep signals the lower face; MDFX_FOLD=0 is
# the two-launch schedule): GPU tests of the engine / proxy / ipc paths, then the proxies A/B.
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=600 scripts/gpu_session.sh "t_fold=python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_proxy.py tests/test_gpu_ipc.py tests/test_gpu_engine.py tests/test_gpu_multiprocess.py" || exit $?
grep -E "passed|failed" gpurun_out/t_fold.log | tail -2
grep -q " failed" gpurun_out/t_fold.log && exit 1
Q="--steps 48 --warmup 5 --graph off --rounds 1 --overlap"
scripts/gpu_session.sh "f8=python bench.py --rank-proxy 8 $Q" "n8=MDFX_FOLD=0 python bench.py --rank-proxy 8 $Q" \
  "f8b=python bench.py --rank-proxy 8 $Q" "n8b=MDFX_FOLD=0 python bench.py --rank-proxy 8 $Q" \
  "f4=python bench.py --rank-proxy 4 $Q" "n4=MDFX_FOLD=0 python bench.py --rank-proxy 4 $Q" \
  "f2=python bench.py --rank-proxy 2 $Q" "n2=MDFX_FOLD=0 python bench.py --rank-proxy 2 $Q" \
  "f8t=python bench.py --rank-proxy 8 --steps 48 --warmup 5" "f4t=python bench.py --rank-proxy 4 --steps 48 --warmup 5" || exit $?
A="--rank-proxy 8 --steps 24 --warmup 4 --graph off --rounds 1 --overlap"
PROF_TAG=f8 BENCH_ARGS="$A" scripts/gpu_session.sh prof || exit $?
for f in f8 n8 f8b n8b f4 n4 f2 n2 f8t f4t; do
  echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
