#!/bin/bash
# Round 5, session T: heat7_wxk K = 5 in fp32 rows of 2 cells per lane (RowOps2f): bitwise against
# the naive kernel on odd shapes, then the 1024^3 kernel A/B against the shipped K = 4.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 200 python bench/kernel_ab.py --kind heat7 --nx 300 --ny 77 --nz 41 --iters 2 --rounds 1 \
  --variants "STEPS=4;STEPS=5;STEPS=5,NAR=1" > $O/ab_odd.log 2>&1 || { tail -20 $O/ab_odd.log; exit 1; }
cat $O/ab_odd.log
timeout -k 10 200 python bench/kernel_ab.py --kind heat7 --nx 1000 --ny 333 --nz 64 --iters 2 --rounds 1 \
  --variants "STEPS=4;STEPS=5;STEPS=5,NAR=1" > $O/ab_odd2.log 2>&1 || { tail -20 $O/ab_odd2.log; exit 1; }
cat $O/ab_odd2.log
timeout -k 10 400 python bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 4 \
  --variants "STEPS=4;STEPS=5;STEPS=5,NAR=1" > $O/ab_1024.log 2>&1 || { tail -20 $O/ab_1024.log; exit 1; }
cat $O/ab_1024.log
