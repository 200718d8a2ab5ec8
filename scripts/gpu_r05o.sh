#!/bin/bash
# Round 5, session O: the headline band with one row fewer in its last wave (2 + 6 x 3 + 1 = 21 rows:
# 245 instead of 235 tiles at 1024^3, A/B switch MDFX_RE2_AB): bitwise tests with the switch on,
# kernel A/B, and the driver form interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05o
mkdir -p $O
MDFX_RE2_AB=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_temporal.py \
  tests/test_gpu_ipc.py -k "heat7_wxk or fp64_fused_k4_folded or multiprocess_matches_single" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 4 \
  --variants "STEPS=4;STEPS=4,RE2=1" > $O/ab_1024.log 2>&1 || { tail -20 $O/ab_1024.log; exit 1; }
tail -3 $O/ab_1024.log
for e in 0 1 0 1 0 1; do
  if [ $e = 1 ]; then export MDFX_RE2_AB=1; else unset MDFX_RE2_AB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_$e.json 2> $O/drv_$e.err || { tail -5 $O/drv_$e.err; exit 1; }
  echo "drv re2=$e $(python -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r['pct_of_measured_copy'], r['config']['verified']['max_abs_diff'])" $O/drv_$e.json)"
done
unset MDFX_RE2_AB
for e in 0 1; do
  if [ $e = 1 ]; then export MDFX_RE2_AB=1; else unset MDFX_RE2_AB; fi
  timeout -k 10 300 python bench.py --rank-proxy 8 --steps 48 --warmup 12 > $O/p8_$e.json 2> $O/p8_$e.err || { tail -5 $O/p8_$e.err; exit 1; }
  echo "proxy8 re2=$e $(grep -o '"value": [0-9.]*' $O/p8_$e.json)"
done
