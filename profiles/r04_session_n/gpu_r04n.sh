#!/bin/bash
# Round 4, session N: box27_wxk band shapes (MDFX_B27_RY), the even sweep plan on the residual
# configs, and the GPU tests of the engine loop.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/n
timeout -k 10 200 python bench/kernel_ab.py --kind box27 --n 512 --dtype f64 --iters 10 --rounds 3 \
  --variants "STEPS=3;STEPS=3,B27RY=1;STEPS=3,B27RY=4" > gpurun_out/n/b27d.log 2>&1 || exit 1
timeout -k 10 200 python bench/kernel_ab.py --kind box27 --n 512 --iters 10 --rounds 3 \
  --variants "STEPS=2;STEPS=3,B27WXK=1;STEPS=3,B27WXK=1,B27RY=1;STEPS=3,B27WXK=1,B27RY=4" > gpurun_out/n/b27f.log 2>&1 || exit 1
tail -4 gpurun_out/n/b27d.log; tail -5 gpurun_out/n/b27f.log
for r in 10 12; do
  timeout -k 10 300 python bench.py --n 2048 --dtype f64 --steps 20 --warmup 2 --residual-every $r \
    > gpurun_out/n/c5_r$r.json 2> gpurun_out/n/c5_r$r.err || { tail -5 gpurun_out/n/c5_r$r.err; exit 1; }
  cat gpurun_out/n/c5_r$r.json
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py tests/test_gpu_temporal.py > gpurun_out/n/gputests.log 2>&1 || { tail -20 gpurun_out/n/gputests.log; exit 1; }
tail -2 gpurun_out/n/gputests.log
