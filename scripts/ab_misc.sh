#!/bin/bash
# Bitwise GPU tests of every stencil kernel, then the benches a shared-helper change touches.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_kernels.py -x 2>&1 | tail -1 || exit 1
b() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['ms_per_step'], d['config'].get('temporal_block'))"; }
echo "== mdf 16384^2 f32"; b --stencil jacobi5 --nx 16384 --nz 16384 --steps 96 --warmup 16 || exit 1
echo "== mdf 16384^2 f64"; b --stencil jacobi5 --dtype f64 --nx 16384 --nz 16384 --steps 96 --warmup 16 || exit 1
echo "== heat7 1024^3"; b || exit 1
echo "== heat7 1024^3 temporal 1"; b --temporal 1 || exit 1
echo "== life 32768^2"; b --stencil life --dtype u8 --nx 32768 --nz 32768 --steps 96 --warmup 12 || exit 1
