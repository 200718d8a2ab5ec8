#!/bin/bash
# Round 5, session F: box27_wxk after the seam-read fix (no window-DMA drain per step), whole-row
# blocks (EXP 16) through the 27-point GPU tests, kernel A/B at 512^3, and the headline after the
# removal of the heat7_wxk A/B copies.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05f
mkdir -p $O
MDFX_WXK_EXP=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py \
  -k "box27_wxk" > $O/t_b27_exp16.log 2>&1 || { tail -20 $O/t_b27_exp16.log; exit 1; }
tail -1 $O/t_b27_exp16.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --iters 10 --rounds 3 \
  --variants "STEPS=2;STEPS=3;STEPS=3,EXP=16" > $O/ab_b27_512_f32.log 2>&1 || { tail -20 $O/ab_b27_512_f32.log; exit 1; }
tail -4 $O/ab_b27_512_f32.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --dtype f64 --iters 10 --rounds 3 \
  --variants "STEPS=3" > $O/ab_b27_512_f64.log 2>&1 || { tail -20 $O/ab_b27_512_f64.log; exit 1; }
tail -2 $O/ab_b27_512_f64.log
timeout -k 10 300 python bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 3 \
  --variants "STEPS=4" > $O/ab_1024.log 2>&1 || { tail -20 $O/ab_1024.log; exit 1; }
tail -2 $O/ab_1024.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_$i.json 2> $O/drv_$i.err || { tail -5 $O/drv_$i.err; exit 1; }
  echo "drv $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], c['verified']['max_abs_diff'])" $O/drv_$i.json)"
done
