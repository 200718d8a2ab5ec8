#!/bin/bash
# Round 3 session E: where heat7_wtk's extra fetch comes from (FETCH_SIZE per row layout and vm
# lag), the ref-precision dispatch, the mdf dialogue, and a kernel-trace timeline of the N=8 proxy.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "ref=$PYT tests/test_gpu_temporal.py -k 'ref_precision or deep_fused'" \
  "dialogue=printf '100\n16384\n16384\n' | ./build/bin/mdf --json" || exit $?
for v in 0 1; do PMC_TAG=nat$v MDFX_WTK_NAT=$v scripts/gpu_session.sh pmc_fetch || exit $?; done
PMC_TAG=lag0 MDFX_VM_LAG=0 scripts/gpu_session.sh pmc_fetch || exit $?
PMC_TAG=dflt scripts/gpu_session.sh pmc_fetch || exit $?
PROF_TAG=proxy8 BENCH_ARGS="--rank-proxy 8 --steps 48 --warmup 12" scripts/gpu_session.sh prof || exit $?
PROF_TAG=proxy8_graphoff BENCH_ARGS="--rank-proxy 8 --steps 48 --warmup 12 --graph off" scripts/gpu_session.sh prof || exit $?
PROF_TAG=h1024 scripts/gpu_session.sh prof || exit $?
tail -n 1 gpurun_out/dialogue.log
