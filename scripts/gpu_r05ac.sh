#!/bin/bash
# Round 5, session AC: K = 5 in 4-wave bands (6 + 4 rows, two blocks per CU: the two blocks'
# plane barriers are independent; MDFX_H7_W4=1) against the shipped 8-wave band.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ac
mkdir -p $O
for shp in "--nx 300 --ny 77 --nz 41" "--nx 1000 --ny 333 --nz 64"; do
  timeout -k 10 200 python bench/kernel_ab.py --kind heat7 $shp --iters 2 --rounds 1 \
    --variants "STEPS=5;STEPS=5,W4=1" > $O/ab_odd.log 2>&1 || { tail -20 $O/ab_odd.log; exit 1; }
  tail -2 $O/ab_odd.log
done
for shp in "--n 1024" "--nx 1024 --ny 1024 --nz 128" "--n 512"; do
  tag=$(echo $shp | tr -d ' -')
  timeout -k 10 300 python bench/kernel_ab.py --kind heat7 $shp --iters 10 --rounds 4 \
    --variants "STEPS=5;STEPS=5,W4=1" > $O/ab_$tag.log 2>&1 || { tail -20 $O/ab_$tag.log; exit 1; }
  echo "== $shp"; tail -2 $O/ab_$tag.log
done
