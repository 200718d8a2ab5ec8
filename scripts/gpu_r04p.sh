#!/bin/bash
# Round 4, session P: fp64 K = 4 through heat7_wxk as the default (fused depth 4 from 1024-cell
# rows) and the cost-based sweep plan: GPU tests of the kernels / engine / ipc / proxy, then the
# fp64 bench configs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/p
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_temporal.py tests/test_gpu_engine.py tests/test_gpu_ipc.py tests/test_gpu_proxy.py \
  > gpurun_out/p/tests.log 2>&1 || { tail -30 gpurun_out/p/tests.log; exit 1; }
tail -2 gpurun_out/p/tests.log
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/p/$tag.json 2> gpurun_out/p/$tag.err || { tail -5 gpurun_out/p/$tag.err; exit 1; }; echo "$tag $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['config']['temporal_block'], d['config'].get('timed_vs_trial'))" gpurun_out/p/$tag.json)"; }
run c5_r12 --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12
run c5_r10 --n 2048 --dtype f64 --steps 20 --warmup 2 --residual-every 10
run c5_proxy8 --rank-proxy 8 --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12
run f64_1024 --n 1024 --dtype f64 --steps 24 --warmup 4
run f64_512 --n 512 --dtype f64 --steps 24 --warmup 4
run f64_512_k4 --n 512 --dtype f64 --steps 24 --warmup 4 --temporal 4
