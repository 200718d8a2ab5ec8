#!/bin/bash
# A/B of the fused 27-point kernels (box27_tb2 vs box27_tbk at RY 2 / 4) after a kernel change;
# bitwise tests first. Output: one line per run.
set -o pipefail
cd "$(dirname "$0")/.."
T="python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -x"
for ry in 2 4; do echo "== box27 tests MDFX_B27_TBK=$ry"; MDFX_B27_TBK=$ry timeout -k 10 300 $T -k "box27 or stale" 2>&1 | tail -1 || exit 1; done
b() { timeout -k 10 200 python bench.py "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', d['value'], d['ms_per_step'], d.get('pct_of_hbm_copy_roof'))"; }
for cfg in "--n 512 --steps 100 --warmup 10" "--n 1024 --steps 20 --warmup 4" "--n 512 --steps 100 --warmup 10 --virtual-ranks 8"; do
for dt in f32 f64; do for ry in 0 2 4; do
  echo "== box27 $cfg $dt MDFX_B27_TBK=$ry"; MDFX_B27_TBK=$ry b --stencil box27 --dtype $dt $cfg || exit 1
done; done; done
