#!/bin/bash
# A/B of the counted vmcnt wait (MDFX_VM_LAG=1: the last plane's output stores stay in flight across
# the next plane's DMA wait) against round 2's vmcnt(0) (MDFX_VM_LAG=0), interleaved, one box.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12"
steps=("temporal=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py")
for r in a b; do
  steps+=("h1024_lag0_$r=MDFX_VM_LAG=0 $B" "h1024_lag1_$r=MDFX_VM_LAG=1 $B")
done
steps+=("v8_lag0=MDFX_VM_LAG=0 $B --virtual-ranks 8" "v8_lag1=MDFX_VM_LAG=1 $B --virtual-ranks 8")
steps+=("h512_lag0=MDFX_VM_LAG=0 $B --n 512" "h512_lag1=MDFX_VM_LAG=1 $B --n 512")
steps+=("b27f32_lag0=MDFX_VM_LAG=0 $B --stencil box27 --n 512" "b27f32_lag1=MDFX_VM_LAG=1 $B --stencil box27 --n 512")
steps+=("b27f64_lag0=MDFX_VM_LAG=0 $B --stencil box27 --n 512 --dtype f64" "b27f64_lag1=MDFX_VM_LAG=1 $B --stencil box27 --n 512 --dtype f64")
steps+=("h1024f64_lag0=MDFX_VM_LAG=0 $B --dtype f64" "h1024f64_lag1=MDFX_VM_LAG=1 $B --dtype f64")
steps+=("drv_lag1=MDFX_VM_LAG=1 python bench.py --steps 20 --warmup 5")
LIMIT=300 scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in gpurun_out/*lag*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
