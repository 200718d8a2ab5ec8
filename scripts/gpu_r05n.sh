#!/bin/bash
# Round 5, session N: the bench with its measured copy yardstick (driver form, 512^3, 27-point, an N = 8
# proxy) and the GPU tests that run bench.py.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05n
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  echo "$tag $(python -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r.get('achieved_dram_TBps_per_gpu', r.get('achieved_dram_TBps')), r.get('measured_copy_TBps'), r.get('pct_of_measured_copy'))" $O/$tag.json)"; }
run driver --gpus 1 --steps 20 --warmup 5
run heat512 --n 512 --steps 100 --warmup 10
run b27_512 --stencil box27 --n 512 --steps 60 --warmup 6
run proxy8 --rank-proxy 8 --steps 48 --warmup 12
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_proxy.py \
  tests/test_gpu_multiprocess.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
