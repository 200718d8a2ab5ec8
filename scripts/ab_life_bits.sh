#!/bin/bash
# Bit-sliced Life (life_bits, default) vs the SWAR kernels: bitwise tests, then 32768^2 sweeps.
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_kernels.py tests/test_gpu_engine.py -k life -x"
timeout -k 10 300 $T 2>&1 | tail -1 || exit 1
b() { timeout -k 10 200 python bench.py --stencil life --dtype u8 --nx 32768 --nz 32768 --steps 96 --warmup 32 "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['ms_per_step'], d['config'].get('temporal_block'))"; }
echo "== swar K=6"; MDFX_LIFE_BITS=0 b --temporal 6 || exit 1
for k in 8 12 16; do for zc in 0 64 128; do
  echo "== bits K=$k zc=$zc"; MDFX_ZC=$zc b --temporal $k || exit 1
done; done
