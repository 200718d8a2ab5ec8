#!/bin/bash
# Round 5, session H: box27_wxk with the held-row / held-plane tests only in the step pairs that need
# them (z-split march), the 27-point GPU tests, the CLI / example tests that now opt in to a shared
# GPU, and the 27-point kernel A/B at 512^3 (fp32, fp64) and 1024^3 fp32.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_cli.py \
  tests/test_examples.py -k "box27 or ipc" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --iters 10 --rounds 3 \
  --variants "STEPS=2;STEPS=3" > $O/ab_b27_512_f32.log 2>&1 || { tail -20 $O/ab_b27_512_f32.log; exit 1; }
tail -3 $O/ab_b27_512_f32.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 512 --dtype f64 --iters 10 --rounds 3 \
  --variants "STEPS=2;STEPS=3" > $O/ab_b27_512_f64.log 2>&1 || { tail -20 $O/ab_b27_512_f64.log; exit 1; }
tail -3 $O/ab_b27_512_f64.log
timeout -k 10 300 python bench/kernel_ab.py --kind box27 --n 1024 --iters 4 --rounds 2 \
  --variants "STEPS=2;STEPS=3" > $O/ab_b27_1024_f32.log 2>&1 || { tail -20 $O/ab_b27_1024_f32.log; exit 1; }
tail -3 $O/ab_b27_1024_f32.log
for d in f32 f64; do
  timeout -k 10 300 python bench.py --stencil box27 --n 512 --dtype $d --steps 60 --warmup 6 > $O/b27_$d.json 2> $O/b27_$d.err || { tail -5 $O/b27_$d.err; exit 1; }
  echo "bench box27 512 $d $(grep -o '"value": [0-9.]*' $O/b27_$d.json)"
done
