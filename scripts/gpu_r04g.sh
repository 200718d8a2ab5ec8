#!/bin/bash
# Round 4 session G: the engine / ipc / proxy GPU tests after dropping the per-step interior event
# (one of them with device-scope sync events), then the N = 8 / 4 proxies and the headline with
# MDFX_EVENT_FENCE=system (HIP default) against device, interleaved; one trace of each at N = 8.
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=500 scripts/gpu_session.sh "t_eng=python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_proxy.py" \
  "t_ipc=MDFX_EVENT_FENCE=device python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ipc.py" || exit $?
grep -E "passed|failed" gpurun_out/t_eng.log gpurun_out/t_ipc.log | tail -2
P8="--rank-proxy 8 --steps 48 --warmup 5 --graph off --rounds 1 --overlap"
P4="--rank-proxy 4 --steps 48 --warmup 5 --graph off --rounds 1 --overlap"
P8P="--rank-proxy 8 --py 2 --steps 48 --warmup 5 --graph off --rounds 1 --overlap"
scripts/gpu_session.sh "p8s=python bench.py $P8" "p8d=MDFX_EVENT_FENCE=device python bench.py $P8" \
  "p8s2=python bench.py $P8" "p8d2=MDFX_EVENT_FENCE=device python bench.py $P8" \
  "p4s=python bench.py $P4" "p4d=MDFX_EVENT_FENCE=device python bench.py $P4" \
  "ps=python bench.py $P8P" "pd=MDFX_EVENT_FENCE=device python bench.py $P8P" \
  "b1s=python bench.py --steps 20 --warmup 5" "b1d=MDFX_EVENT_FENCE=device python bench.py --steps 20 --warmup 5" || exit $?
A="--rank-proxy 8 --steps 24 --warmup 4 --graph off --rounds 1 --overlap"
PROF_TAG=p8s BENCH_ARGS="$A" scripts/gpu_session.sh prof || exit $?
(export MDFX_EVENT_FENCE=device; PROF_TAG=p8d BENCH_ARGS="$A" scripts/gpu_session.sh prof) || exit $?
for f in p8s p8d p8s2 p8d2 p4s p4d ps pd b1s b1d; do
  echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
