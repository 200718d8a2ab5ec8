#!/bin/bash
# Round 4, session R: fp32 K = 4 heat7_wxk band shapes (MDFX_WXK_SHAPE experiment: 3 + 1 and
# 2 + 1-row bands against the shipped 3 + 2) at 1024^3 and 512^3, kernel A/B and the driver bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r
for n in 1024 512; do
  timeout -k 10 300 python bench/kernel_ab.py --kind heat7 --n $n --iters 10 --rounds 3 \
    --variants "STEPS=4;STEPS=4,SHAPE=1;STEPS=4,SHAPE=2;STEPS=4" > gpurun_out/r/ab_$n.log 2>&1 || { tail -20 gpurun_out/r/ab_$n.log; exit 1; }
  tail -5 gpurun_out/r/ab_$n.log
done
for sh in 0 1 2; do
  MDFX_WXK_SHAPE=$sh timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r/drv_$sh.json 2> gpurun_out/r/drv_$sh.err || { tail -5 gpurun_out/r/drv_$sh.err; exit 1; }
  echo "shape $sh $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" gpurun_out/r/drv_$sh.json)"
done
