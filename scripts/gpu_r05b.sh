#!/bin/bash
# Round 5, session B: heat7_wxk (LDS reads now hoisted in every copy) with non-temporal window DMAs
# (EXP 1), an L2 prefetch of plane q + 2 issued outside the compiler's view (EXP 2), the z-test-free
# middle of the march (EXP 4) and combinations; box27_wxk with nt DMAs; driver-form bench.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 400 python bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 4 \
  --variants "STEPS=4;STEPS=4,EXP=1;STEPS=4,EXP=2;STEPS=4,EXP=4;STEPS=4,EXP=5;STEPS=4,EXP=7" > $O/ab_1024.log 2>&1 || { tail -20 $O/ab_1024.log; exit 1; }
tail -8 $O/ab_1024.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --dtype f64 --iters 10 --rounds 3 \
  --variants "STEPS=3;STEPS=3,EXP=1" > $O/ab_b27_512_f64.log 2>&1 || { tail -20 $O/ab_b27_512_f64.log; exit 1; }
tail -3 $O/ab_b27_512_f64.log
for e in 0 1 4 5 0 1 4 5; do
  MDFX_WXK_EXP=$e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_$e.json 2> $O/drv_$e.err || { tail -5 $O/drv_$e.err; exit 1; }
  echo "exp $e $(python -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r['config']['verified']['max_abs_diff'])" $O/drv_$e.json)"
done
