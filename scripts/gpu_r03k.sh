#!/bin/bash
# Round 3 session K: what bounds heat7_wxk K = 4 (SQ counters, LDS bank conflicts), the 3 + 2 band
# for tile rounding on thin slabs, and the N = 8 proxy timeline.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "wxk=$PYT tests/test_gpu_temporal.py -k 'wxk'" || exit $?
grep -q ' passed' gpurun_out/wxk.log && ! grep -q 'failed' gpurun_out/wxk.log || { tail -30 gpurun_out/wxk.log; exit 1; }
B="python bench.py --steps 48 --warmup 12"
P8="python bench.py --rank-proxy 8 --steps 48 --warmup 12"
scripts/gpu_session.sh "d=$B" "r32=MDFX_WXK_RY=32 $B" "p8=$P8" "p8r32=MDFX_WXK_RY=32 $P8" "p8r31=MDFX_WXK_RY=31 $P8" \
  "p4=python bench.py --rank-proxy 4 --steps 48 --warmup 12" "p4r32=MDFX_WXK_RY=32 python bench.py --rank-proxy 4 --steps 48 --warmup 12" || exit $?
TAG=wxk4 bash scripts/pmc_sq.sh || exit $?
TAG=wxk4lds CTRS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA" bash scripts/pmc_sq.sh || exit $?
PROF_TAG=p8k4 BENCH_ARGS="--rank-proxy 8 --steps 48 --warmup 12" scripts/gpu_session.sh prof || exit $?
for f in d r32 p8 p8r32 p8r31 p4 p4r32; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
