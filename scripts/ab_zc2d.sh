#!/bin/bash
# z-chunk (rows per wave task) sweep of the deep 2D kernels: each chunk recomputes 2K fill rows.
cd "$(dirname "$0")/.."
b() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['ms_per_step'], d['config'].get('temporal_block'))"; }
for k in 4 6 8; do for zc in 0 64 128 256; do
  echo "== life K=$k zc=$zc"; MDFX_ZC=$zc b --stencil life --dtype u8 --nx 32768 --nz 32768 --steps 96 --warmup 12 --temporal $k || exit 1
done; done
for zc in 0 256; do echo "== mdf K=8 zc=$zc"; MDFX_ZC=$zc b --stencil jacobi5 --nx 16384 --nz 16384 --steps 96 --warmup 16 || exit 1; done
