#!/bin/bash
# Round 4 session K: the upper boundary launch signals the fold counter (no boundary event), 2-wave
# strip chunks down to K planes: GPU tests, slab A/B against the two-launch schedule, pencil proxies.
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=600 scripts/gpu_session.sh "t_k=python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_proxy.py tests/test_gpu_ipc.py tests/test_gpu_engine.py tests/test_gpu_multiprocess.py" || exit $?
grep -E "passed|failed" gpurun_out/t_k.log | tail -1
grep -q " failed" gpurun_out/t_k.log && exit 1
Q="--steps 48 --warmup 5 --graph off --rounds 1 --overlap"
scripts/gpu_session.sh "f8=python bench.py --rank-proxy 8 $Q" "n8=MDFX_FOLD=0 python bench.py --rank-proxy 8 $Q" \
  "f8b=python bench.py --rank-proxy 8 $Q" "n8b=MDFX_FOLD=0 python bench.py --rank-proxy 8 $Q" \
  "f4=python bench.py --rank-proxy 4 $Q" "n4=MDFX_FOLD=0 python bench.py --rank-proxy 4 $Q" \
  "s8=python bench.py --rank-proxy 8 --py 2 $Q" "o8=MDFX_WXK_STRIP=0 python bench.py --rank-proxy 8 --py 2 $Q" \
  "f8t=python bench.py --rank-proxy 8 --steps 48 --warmup 5" "f4t=python bench.py --rank-proxy 4 --steps 48 --warmup 5" \
  "f2t=python bench.py --rank-proxy 2 --steps 48 --warmup 5" "s8t=python bench.py --rank-proxy 8 --py 2 --steps 48 --warmup 5" \
  "b1=python bench.py --steps 20 --warmup 5" || exit $?
A="--rank-proxy 8 --steps 24 --warmup 4 --graph off --rounds 1 --overlap"
PROF_TAG=f8 BENCH_ARGS="$A" scripts/gpu_session.sh prof || exit $?
PROF_TAG=s8 BENCH_ARGS="$A --py 2" scripts/gpu_session.sh prof || exit $?
for f in f8 n8 f8b n8b f4 n4 s8 o8 f8t f4t f2t s8t b1; do
  echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
