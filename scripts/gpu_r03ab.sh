#!/bin/bash
# Round 3 session AB: jacobi5_tbk rows in flight: mode 2 (two, default) vs mode 3 (four, occupancy 2)
# vs mode 1 (one), 16384^2 fp32, two passes; the 2D bitwise tier under mode 3.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "tj5m3=MDFX_J5_NAT=3 $PYT tests/test_gpu_temporal.py tests/test_gpu_kernels.py -k 'mdf or jacobi5 or deep or 2d'" || exit $?
grep -q ' passed' gpurun_out/tj5m3.log && ! grep -q 'failed' gpurun_out/tj5m3.log || { tail -30 gpurun_out/tj5m3.log; exit 1; }
B="python bench.py --stencil jacobi5 --nx 16384 --nz 16384 --steps 96 --warmup 16"
scripts/gpu_session.sh "m2a=$B" "m3a=MDFX_J5_NAT=3 $B" "m1a=MDFX_J5_NAT=1 $B" "m2b=$B" "m3b=MDFX_J5_NAT=3 $B" "m1b=MDFX_J5_NAT=1 $B" || exit $?
for f in m2a m3a m1a m2b m3b m1b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep -E 'passed|failed' gpurun_out/tj5m3.log | tail -1
