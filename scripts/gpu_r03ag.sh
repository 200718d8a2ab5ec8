#!/bin/bash
# Round 3 session AG: fused depth for the thin N = 8 slab (1024^2 x 128): K = 4 (default) vs 3 vs 2, rank proxy, twice each.
set -o pipefail
cd "$(dirname "$0")/.."
P="python bench.py --steps 48 --warmup 12 --rank-proxy 8"
scripts/gpu_session.sh "k4a=$P" "k3a=$P --temporal 3" "k2a=$P --temporal 2" "k4b=$P" "k3b=$P --temporal 3" "k2b=$P --temporal 2" || exit $?
for f in k4a k3a k2a k4b k3b k2b; do echo "$f $(grep -o '"value": [0-9.]*\|"temporal_block": [0-9]*' gpurun_out/$f.log | tr '\n' ' ')"; done
