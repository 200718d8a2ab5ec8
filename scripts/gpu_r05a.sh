#!/bin/bash
# Round 5, session A: LDS reads hoisted to the top of each plane step (MDFX_WXK_EXP=1) in heat7_wxk
# and box27_wxk against the shipped kernels; the x-balance probe (nx = 992: 4 x segments, 188 tiles
# instead of 235); the driver-form bench (with the new timed-run verification).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 300 python bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 4 \
  --variants "STEPS=4;STEPS=4,EXP=1;STEPS=4,EXP=3;STEPS=4;STEPS=4,EXP=1" > $O/ab_1024.log 2>&1 || { tail -20 $O/ab_1024.log; exit 1; }
tail -6 $O/ab_1024.log
timeout -k 10 300 python bench/kernel_ab.py --kind heat7 --nx 992 --ny 1024 --nz 1024 --iters 10 --rounds 3 \
  --variants "STEPS=4;STEPS=4,EXP=1;STEPS=4,EXP=3" > $O/ab_992.log 2>&1 || { tail -20 $O/ab_992.log; exit 1; }
tail -4 $O/ab_992.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --iters 10 --rounds 3 \
  --variants "STEPS=2;STEPS=3;STEPS=3,EXP=1" > $O/ab_b27_512_f32.log 2>&1 || { tail -20 $O/ab_b27_512_f32.log; exit 1; }
tail -5 $O/ab_b27_512_f32.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --dtype f64 --iters 10 --rounds 3 \
  --variants "STEPS=3;STEPS=3,EXP=1" > $O/ab_b27_512_f64.log 2>&1 || { tail -20 $O/ab_b27_512_f64.log; exit 1; }
tail -4 $O/ab_b27_512_f64.log
for e in 0 1 0 1; do
  MDFX_WXK_EXP=$e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_$e.json 2> $O/drv_$e.err || { tail -5 $O/drv_$e.err; exit 1; }
  echo "exp $e $(python -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r['config']['verified'])" $O/drv_$e.json)"
done
