#!/bin/bash
# Round 3 session AJ: fresh engine for the timed run after the trials (proxy and N > 1): proxy K = 2 graph on,
# proxy default, bench / proxy GPU tests, torchrun N = 2 sharing the GPU.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
P="python bench.py --steps 48 --warmup 12 --rank-proxy 8"
scripts/gpu_session.sh "aj_k2g=$P --temporal 2 --graph on --rounds 2" "aj_p8=$P" "aj_tests=$PYT tests/test_gpu_proxy.py tests/test_gpu_multiprocess.py" || exit $?
grep -q ' passed' gpurun_out/aj_tests.log && ! grep -q 'failed' gpurun_out/aj_tests.log || { tail -30 gpurun_out/aj_tests.log; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29502 \
  bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 --timeout 60 > gpurun_out/aj_torchrun_2.log 2>&1 || { tail -30 gpurun_out/aj_torchrun_2.log; exit 1; }
for f in aj_k2g aj_p8 aj_torchrun_2; do echo "$f $(grep -o '"value": [0-9.]*\|"graph": [a-z]*' gpurun_out/$f.log | head -2 | tr '\n' ' ')"; done
grep -E 'passed|failed' gpurun_out/aj_tests.log | tail -1
