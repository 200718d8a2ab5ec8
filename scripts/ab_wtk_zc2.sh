#!/bin/bash
# heat7_wtk z chunks on the single-slab shapes of the N = 2 / 4 runs (1024 x 1024 x nz, one rank):
# automatic vs chunk counts whose last round of blocks is nearly full.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
LIMIT=300 scripts/gpu_session.sh \
  "z2_512_auto=$B --nx 1024 --ny 1024 --nz 512" "z2_512_73=MDFX_ZC=73 $B --nx 1024 --ny 1024 --nz 512" \
  "z2_512_86=MDFX_ZC=86 $B --nx 1024 --ny 1024 --nz 512" "z2_512_43=MDFX_ZC=43 $B --nx 1024 --ny 1024 --nz 512" \
  "z2_256_auto=$B --nx 1024 --ny 1024 --nz 256" "z2_256_37=MDFX_ZC=37 $B --nx 1024 --ny 1024 --nz 256" \
  "z2_256_43=MDFX_ZC=43 $B --nx 1024 --ny 1024 --nz 256" "z2_512_autob=$B --nx 1024 --ny 1024 --nz 512" \
  "z2_512_73b=MDFX_ZC=73 $B --nx 1024 --ny 1024 --nz 512" || exit $?
for f in gpurun_out/z2_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
