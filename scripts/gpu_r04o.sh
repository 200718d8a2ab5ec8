#!/bin/bash
# Round 4, session O: fp64 K = 4 through heat7_wxk (2 + 1-row bands, MDFX_WXK_F64K4=1) against
# heat7_wtk K = 4 and the shipped fp64 K = 3: bitwise tests, kernel A/B, bench configs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_temporal.py -k "wxk" > gpurun_out/o/tests.log 2>&1 || { tail -30 gpurun_out/o/tests.log; exit 1; }
tail -2 gpurun_out/o/tests.log
for n in 1024; do  # (2048^3 fp64: kernel_ab's fields do not fit; the bench below covers it)
  timeout -k 10 300 python bench/kernel_ab.py --kind heat7 --n $n --dtype f64 --iters 6 --rounds 3 \
    --variants "STEPS=3;STEPS=4;STEPS=4,F64K4=1,WXK=1;STEPS=3,WXK=1" > gpurun_out/o/ab_$n.log 2>&1 || { tail -20 gpurun_out/o/ab_$n.log; exit 1; }
  tail -5 gpurun_out/o/ab_$n.log
done
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/o/$tag.json 2> gpurun_out/o/$tag.err || { tail -5 gpurun_out/o/$tag.err; exit 1; }; echo "$tag $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['config']['temporal_block'])" gpurun_out/o/$tag.json)"; }
run r12_k3 --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12
MDFX_WXK_F64K4=1 run r12_k4 --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12 --temporal 4
run f64_1024_k3 --n 1024 --dtype f64 --steps 24 --warmup 4
MDFX_WXK_F64K4=1 MDFX_H7_WXK=1 run f64_1024_k4 --n 1024 --dtype f64 --steps 24 --warmup 4 --temporal 4
