#!/bin/bash
# heat7_wtk z-chunk sweep (MDFX_ZC) at 1024^3 fp32 K = 3 (bands of 8) and on the 8-slab shape.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
steps=("zc_auto_a=$B")
for zc in 64 128 171 256 342 512; do steps+=("zc_${zc}=MDFX_ZC=$zc $B"); done
steps+=("zc_auto_b=$B" "zcv8_auto=$B --virtual-ranks 8")
for zc in 32 43 64; do steps+=("zcv8_${zc}=MDFX_ZC=$zc $B --virtual-ranks 8"); done
LIMIT=300 scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in gpurun_out/zc*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
