#!/bin/bash
set -o pipefail
cd /root/repo
export MDFX_H7_WTK=1 MDFX_WTK_RY=3
PMC_TAG=wtk3 BENCH_ARGS="--temporal 3" scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
TAG=wtk3 BENCH_ARGS="--temporal 3" bash scripts/pmc_sq.sh || exit $?
unset MDFX_H7_WTK MDFX_WTK_RY
TAG=tbk2 BENCH_ARGS="--temporal 2" bash scripts/pmc_sq.sh || exit $?
python3 scripts/pmc_sq_summary.py gpurun_out/sq_wtk3 gpurun_out/sq_tbk2 > gpurun_out/sq_summary.txt
