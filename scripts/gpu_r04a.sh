#!/bin/bash
# Round 4 session A: SDMA (NoCU) face copies and the direct ipc pull against round 3's blit + mailbox
# exchange in the rank proxies; proxy / ipc tests on the new paths; the headline bench; SQ counters
# of the shipped heat7_wxk sweep; a kernel trace of the N = 8 proxy.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "proxy_t=$PYT tests/test_gpu_proxy.py" "ipc_t=$PYT tests/test_gpu_ipc.py" || exit $?
B="python bench.py --steps 20 --warmup 5"
P8="python bench.py --rank-proxy 8 --steps 48 --warmup 5"
P4="python bench.py --rank-proxy 4 --steps 48 --warmup 5"
scripts/gpu_session.sh "drv=$B" "p8_old=MDFX_XCOPY=blit MDFX_IPC_DIRECT=0 $P8" "p8_sdma_mbox=MDFX_IPC_DIRECT=0 $P8" \
  "p8=$P8" "p8_blit_direct=MDFX_XCOPY=blit $P8" "p4_old=MDFX_XCOPY=blit MDFX_IPC_DIRECT=0 $P4" "p4=$P4" || exit $?
PROF_TAG=p8 BENCH_ARGS="--rank-proxy 8 --steps 48 --warmup 5" scripts/gpu_session.sh prof || exit $?
TAG=wxk4 BENCH_ARGS="--temporal 4" bash scripts/pmc_sq.sh || exit $?
TAG=wxk4lds CTRS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA" BENCH_ARGS="--temporal 4" bash scripts/pmc_sq.sh || exit $?
TAG=wxk4vm CTRS="SQ_WAVES SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY" BENCH_ARGS="--temporal 4" bash scripts/pmc_sq.sh || exit $?
for f in drv p8_old p8_sdma_mbox p8 p8_blit_direct p4_old p4; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"timed_vs_trial": [0-9.a-z]*' gpurun_out/$f.log)"; done
