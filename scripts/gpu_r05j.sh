#!/bin/bash
# Round 5, session J: heat7_wxk whole-row blocks (2 x 4 waves, LDS x edges) for fp32 rows <= 512
# (A/B switch MDFX_XW_AB): the bitwise tests with the switch on, kernel A/B at 512^3, bench form.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05j
mkdir -p $O
MDFX_XW_AB=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_temporal.py \
  -k "heat7_wxk" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench/kernel_ab.py --kind heat7 --n 512 --iters 10 --rounds 3 \
  --variants "STEPS=4;STEPS=4,XW=1" > $O/ab_512.log 2>&1 || { tail -20 $O/ab_512.log; exit 1; }
tail -3 $O/ab_512.log
for e in 0 1 0 1; do
  if [ $e = 1 ]; then export MDFX_XW_AB=1; else unset MDFX_XW_AB; fi
  timeout -k 10 300 python bench.py --n 512 --steps 100 --warmup 10 > $O/b512_$e.json 2> $O/b512_$e.err || { tail -5 $O/b512_$e.err; exit 1; }
  echo "bench 512 xw=$e $(grep -o '"value": [0-9.]*' $O/b512_$e.json) $(grep -o '"max_abs_diff": [0-9.e-]*' $O/b512_$e.json)"
done
