#!/bin/bash
# Round 4, session Y: the z-trapezoid fill of heat7_wxk (working tree) against HEAD without it
# (ab_alt/, scripts/make_ab_alt.sh), interleaved on one box: bitwise wxk tests first.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/y
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py -k "wxk or fp64" \
  > gpurun_out/y/tests.log 2>&1 || { tail -30 gpurun_out/y/tests.log; exit 1; }
tail -1 gpurun_out/y/tests.log
for rep in 1 2; do
  for tree in new old; do
    kab=bench/kernel_ab.py; [ $tree = old ] && kab=ab_alt/bench/kernel_ab.py
    timeout -k 10 200 python $kab --kind heat7 --n 1024 --iters 10 --rounds 3 --variants "STEPS=4" > gpurun_out/y/f32_${tree}_$rep.log 2>&1 || { tail -5 gpurun_out/y/f32_${tree}_$rep.log; exit 1; }
    timeout -k 10 200 python $kab --kind heat7 --n 1024 --dtype f64 --iters 6 --rounds 3 --variants "STEPS=4" > gpurun_out/y/f64_${tree}_$rep.log 2>&1 || { tail -5 gpurun_out/y/f64_${tree}_$rep.log; exit 1; }
    echo "$tree rep$rep f32 $(grep '^STEPS=4' gpurun_out/y/f32_${tree}_$rep.log | head -1)"
    echo "$tree rep$rep f64 $(grep '^STEPS=4' gpurun_out/y/f64_${tree}_$rep.log | head -1)"
  done
done
for tree in new old; do
  b=bench.py; [ $tree = old ] && b=ab_alt/bench.py
  timeout -k 10 200 python $b --rank-proxy 8 --steps 48 --warmup 12 > gpurun_out/y/p8_$tree.json 2>/dev/null || exit 1
  timeout -k 10 200 python $b --gpus 1 --steps 20 --warmup 5 > gpurun_out/y/drv_$tree.json 2>/dev/null || exit 1
  echo "$tree p8 $(grep -o '"value": [0-9.]*' gpurun_out/y/p8_$tree.json) drv $(grep -o '"value": [0-9.]*' gpurun_out/y/drv_$tree.json)"
done
