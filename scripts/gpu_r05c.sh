#!/bin/bash
# Round 5, session C: the window DMA two planes ahead in the same two buffers (EXP 8) and with the
# z-test-free march middle (EXP 12) against the hoisted default, kernel A/B with a fresh grid per
# variant and the driver-form bench interleaved; box27_tb2n with hoisted seam reads (EXP 8).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 400 python bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 4 \
  --variants "STEPS=4;STEPS=4,EXP=8;STEPS=4,EXP=4;STEPS=4,EXP=12" > $O/ab_1024.log 2>&1 || { tail -20 $O/ab_1024.log; exit 1; }
tail -6 $O/ab_1024.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --iters 10 --rounds 3 \
  --variants "STEPS=2;STEPS=2,EXP=8;STEPS=3" > $O/ab_b27_512_f32.log 2>&1 || { tail -20 $O/ab_b27_512_f32.log; exit 1; }
tail -4 $O/ab_b27_512_f32.log
for e in 0 8 12 0 8 12 0 8; do
  MDFX_WXK_EXP=$e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_$e.json 2> $O/drv_$e.err || { tail -5 $O/drv_$e.err; exit 1; }
  echo "exp $e $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], c['verified']['max_abs_diff'], [(t['graph'], t['ms_per_step']) for t in c['trials']])" $O/drv_$e.json)"
done
