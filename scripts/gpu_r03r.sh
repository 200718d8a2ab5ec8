#!/bin/bash
# Round 3 session R: heat7_wxk window depth (u0 DMA 2 planes ahead, 3 window buffers) and the
# single seam table (2 barriers per plane) against the shipped 3+2 band; fp64 2048^3 without a
# residual (heat7_wxk 3+1 default vs heat7_wtk); the staged-fallback bench test.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "tdepth=$PYT tests/test_gpu_temporal.py -k 'window_depth or fp64_wide or wxk_bitwise'" \
  "tdepth_eng=MDFX_WXK_NB=31 $PYT tests/test_gpu_temporal.py -k 'wxk_regions_and_engine'" \
  "fallback=$PYT tests/test_gpu_multiprocess.py -k 'fallback'" || exit $?
for f in tdepth tdepth_eng fallback; do grep -q ' passed' gpurun_out/$f.log && ! grep -q 'failed' gpurun_out/$f.log || { tail -30 gpurun_out/$f.log; exit 1; }; done
B="python bench.py --steps 48 --warmup 12"
P="python bench.py --steps 48 --warmup 12 --rank-proxy 8"
steps=()
for pass in a b; do
  steps+=("d_$pass=$B" "nb31_$pass=MDFX_WXK_NB=31 $B" "nb21_$pass=MDFX_WXK_NB=21 $B" "nb32_$pass=MDFX_WXK_NB=32 $B")
done
steps+=("p8=$P" "p8nb31=MDFX_WXK_NB=31 $P" "drv=python bench.py --steps 20 --warmup 5" "drv31=MDFX_WXK_NB=31 python bench.py --steps 20 --warmup 5")
F="python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3"
steps+=("f64n_wxk=$F" "f64n_wtk=MDFX_H7_WXK=0 $F")
scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in d_a nb31_a nb21_a nb32_a d_b nb31_b nb21_b nb32_b p8 p8nb31 drv drv31 f64n_wxk f64n_wtk; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
