#!/bin/bash
# Life kernels after a change: bitwise tests, then 32768^2 sweeps at every fused depth.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_kernels.py tests/test_gpu_engine.py -k "life or Life" -x 2>&1 | tail -2 || exit 1
b() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['ms_per_step'], d['config'].get('temporal_block'))"; }
for k in auto 1 2 4 6 8; do
  echo "== life 32768^2 temporal $k"; b --stencil life --dtype u8 --nx 32768 --nz 32768 --steps 100 --warmup 10 $([[ $k != auto ]] && echo --temporal $k) || exit 1
done
