#!/bin/bash
# Round 3 session AA: jacobi5_tbk (2D MDF, fp32 natural layout) with two u0 rows in flight instead of
# one: the 2D bitwise tier, then 16384^2 fp32 against mode 1, and the reference's dialogue.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "tj5=$PYT tests/test_gpu_temporal.py tests/test_gpu_kernels.py tests/test_gpu_engine.py -k 'mdf or jacobi5 or deep or 2d'" || exit $?
grep -q ' passed' gpurun_out/tj5.log && ! grep -q 'failed' gpurun_out/tj5.log || { tail -30 gpurun_out/tj5.log; exit 1; }
B="python bench.py --stencil jacobi5 --nx 16384 --nz 16384 --steps 96 --warmup 16"
scripts/gpu_session.sh "m2a=$B" "m1a=MDFX_J5_NAT=1 $B" "m2b=$B" "m1b=MDFX_J5_NAT=1 $B" "m2ref=$B --ref-precision" "m2f64=$B --dtype f64" || exit $?
for i in 1 2; do printf '100\n16384\n16384\n' | timeout -k 10 120 ./build/bin/mdf --json > gpurun_out/dlg_$i.json 2>&1 || exit 1; done
for f in m2a m1a m2b m1b m2ref m2f64; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
for i in 1 2; do echo "dialogue_$i $(grep -o '"value": [0-9.]*' gpurun_out/dlg_$i.json)"; done
grep -E 'passed|failed' gpurun_out/tj5.log | tail -1
