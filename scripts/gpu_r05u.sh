#!/bin/bash
# Round 5, session U: heat7_wxk K = 5 (2-cell lanes) against K = 4 / 3 at other shapes: 512^3,
# 2048^2 x 512, and the slabs of the N = 4 / 8 proxies (1024^2 x 256 / 128).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05u
mkdir -p $O
for shp in "--n 512" "--nx 2048 --ny 2048 --nz 512" "--nx 1024 --ny 1024 --nz 256" "--nx 1024 --ny 1024 --nz 128" "--nx 768 --ny 768 --nz 768"; do
  tag=$(echo $shp | tr -d ' -')
  timeout -k 10 300 python bench/kernel_ab.py --kind heat7 $shp --iters 10 --rounds 3 \
    --variants "STEPS=3;STEPS=4;STEPS=5" > $O/ab_$tag.log 2>&1 || { tail -20 $O/ab_$tag.log; exit 1; }
  echo "== $shp"; tail -4 $O/ab_$tag.log
done
