#!/bin/bash
# 2D MDF kernels after a change: bitwise tests, then 16384^2 fp32 / fp64 at the automatic depth.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_kernels.py tests/test_gpu_engine.py -k "mdf or jacobi5 or deep or stale" -x 2>&1 | tail -1 || exit 1
b() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['ms_per_step'], d['config'].get('temporal_block'))"; }
for dt in f32 f64; do for i in 1 2; do echo "== mdf 16384^2 $dt"; b --stencil jacobi5 --dtype $dt --nx 16384 --nz 16384 --steps 96 --warmup 16 || exit 1; done; done
