#!/bin/bash
# Bands of 4 vs 8 waves on one GPU holding a single slab of the N = 2 / 4 / 8 shapes
# (1024 x 1024 x nz, one rank): what each GPU of a one-process-per-GPU run computes.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on --temporal 3"
steps=()
for nz in 512 256 128; do for wb in 4 8; do steps+=("wb_nz${nz}_wb$wb=MDFX_WTK_WB=$wb $B --nx 1024 --ny 1024 --nz $nz"); done; done
LIMIT=300 scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in gpurun_out/wb_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
