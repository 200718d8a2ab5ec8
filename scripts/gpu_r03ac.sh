#!/bin/bash
# Round 3 session AC: fp64 jacobi5_tbk with two u0 rows in flight (MDFX_J5_F64_PD=1) vs mode 0.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "tj5f64=MDFX_J5_F64_PD=1 $PYT tests/test_gpu_temporal.py tests/test_gpu_kernels.py -k 'mdf or jacobi5 or deep or 2d'" || exit $?
grep -q ' passed' gpurun_out/tj5f64.log && ! grep -q 'failed' gpurun_out/tj5f64.log || { tail -30 gpurun_out/tj5f64.log; exit 1; }
B="python bench.py --stencil jacobi5 --dtype f64 --nx 16384 --nz 16384 --steps 96 --warmup 16"
scripts/gpu_session.sh "d0a=$B" "d1a=MDFX_J5_F64_PD=1 $B" "d0b=$B" "d1b=MDFX_J5_F64_PD=1 $B" || exit $?
for f in d0a d1a d0b d1b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep -E 'passed|failed' gpurun_out/tj5f64.log | tail -1
