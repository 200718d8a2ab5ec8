#!/bin/bash
# Round 5, session G3: the captured-graph fold check, one FETCH_SIZE and one WRITE_SIZE pass per
# shipped 27-point instance at 512^3, and every BASELINE config that fits one MI355X.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh "gfold=python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_ipc.py -k fp64_fused_k4_folded" || exit $?
grep -E "passed|failed" gpurun_out/gfold.log | tail -1
PMC_TAG=b27f32 BENCH_ARGS="--stencil box27 --n 512" scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
PMC_TAG=b27f64 BENCH_ARGS="--stencil box27 --n 512 --dtype f64" scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
LIMIT=900 scripts/gpu_session.sh "baseline=bash scripts/baseline_configs.sh" || exit $?
for f in gpurun_out/baseline_*.json; do echo "$(basename $f .json) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
