#!/bin/bash
# z-chunk / rows-per-tile sweeps for the x-tiled fp64 7-point (2048^3) and the fused 27-point (512^3).
B="python bench.py --graph off"
F="$B --n 2048 --dtype f64 --residual-every 10 --steps 20 --warmup 4"
X="$B --stencil box27 --n 512 --steps 48 --warmup 8"
LIMIT=150 bash "$(dirname "$0")/gpu_session.sh" \
 "f64_zc0=$F" "f64_zc16=MDFX_ZC=16 $F" "f64_zc24=MDFX_ZC=24 $F" "f64_zc32=MDFX_ZC=32 $F" "f64_zc64=MDFX_ZC=64 $F" \
 "b27_zc0=$X" "b27_zc16=MDFX_ZC=16 $X" "b27_zc32=MDFX_ZC=32 $X" "b27_zc64=MDFX_ZC=64 $X" "b27_ry1=MDFX_TB_RY=1 $X" \
 "b27d_zc0=$X --dtype f64" "b27d_zc16=MDFX_ZC=16 $X --dtype f64" "b27d_zc32=MDFX_ZC=32 $X --dtype f64" "b27d_ry1=MDFX_TB_RY=1 $X --dtype f64"
