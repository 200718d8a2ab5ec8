#!/bin/bash
# Round 3 session X: boundary kernels on the compute stream (MDFX_BND_CS=1, new default) -- the
# engine / proxy / ipc / multi-process tiers, then rank proxies, 8 virtual slabs and 2 ipc
# processes against MDFX_BND_CS=0, and the headline.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "teng=$PYT tests/test_gpu_engine.py tests/test_gpu_proxy.py tests/test_gpu_multiprocess.py tests/test_gpu_temporal.py -k 'engine or proxy or multiprocess or regions or slab or graph or overlap'" ipc || exit $?
for f in teng ipc; do grep -q ' passed' gpurun_out/$f.log && ! grep -q 'failed' gpurun_out/$f.log || { tail -30 gpurun_out/$f.log; exit 1; }; done
P="python bench.py --steps 48 --warmup 12 --rank-proxy"
steps=()
for pass in a b; do
  for n in 8 4 2; do steps+=("p${n}_cs1_$pass=$P $n" "p${n}_cs0_$pass=MDFX_BND_CS=0 $P $n"); done
done
B="python bench.py --steps 48 --warmup 12"
steps+=("v8_cs1=$B --virtual-ranks 8" "v8_cs0=MDFX_BND_CS=0 $B --virtual-ranks 8" "ipc2_cs1=$B --gpus 2 --share-gpu --transport ipc" "ipc2_cs0=MDFX_BND_CS=0 $B --gpus 2 --share-gpu --transport ipc" "h1=$B")
scripts/gpu_session.sh "${steps[@]}" || exit $?
PROF_TAG=p8cs1 BENCH_ARGS="--steps 48 --warmup 12 --rank-proxy 8 --graph off --rounds 1" scripts/gpu_session.sh prof || exit $?
python3 scripts/kernel_timeline.py gpurun_out/prof_p8cs1 --skip 200 > gpurun_out/timeline_p8cs1.txt 2>&1
for f in p8_cs1_a p8_cs0_a p4_cs1_a p4_cs0_a p2_cs1_a p2_cs0_a p8_cs1_b p8_cs0_b p4_cs1_b p4_cs0_b p2_cs1_b p2_cs0_b v8_cs1 v8_cs0 ipc2_cs1 ipc2_cs0 h1; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep -E 'passed|failed' gpurun_out/teng.log | tail -1
