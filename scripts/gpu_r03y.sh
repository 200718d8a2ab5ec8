#!/bin/bash
# Round 3 session Y: fused boundary + interior launch (MDFX_BND_FUSE=1, new default for the middle
# ranks): ipc / proxy / engine / multi-process tiers, then rank proxies and the headline against
# MDFX_BND_FUSE=0.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh ipc "teng=$PYT tests/test_gpu_engine.py tests/test_gpu_proxy.py tests/test_gpu_multiprocess.py tests/test_gpu_temporal.py -k 'engine or proxy or multiprocess or regions or slab or graph or overlap or wxk'" || exit $?
for f in teng ipc; do grep -q ' passed' gpurun_out/$f.log && ! grep -q 'failed' gpurun_out/$f.log || { tail -30 gpurun_out/$f.log; exit 1; }; done
P="python bench.py --steps 48 --warmup 12 --rank-proxy"
steps=()
for pass in a b; do
  for n in 8 4 2; do steps+=("p${n}_f1_$pass=$P $n" "p${n}_f0_$pass=MDFX_BND_FUSE=0 $P $n"); done
done
B="python bench.py --steps 48 --warmup 12"
steps+=("ipc3_f1=$B --gpus 3 --share-gpu --transport ipc" "ipc3_f0=MDFX_BND_FUSE=0 $B --gpus 3 --share-gpu --transport ipc" "h1=$B" "hdrv=python bench.py --steps 20 --warmup 5")
scripts/gpu_session.sh "${steps[@]}" || exit $?
PROF_TAG=p8f1 BENCH_ARGS="--steps 48 --warmup 12 --rank-proxy 8 --graph off --rounds 1" scripts/gpu_session.sh prof || exit $?
for f in p8_f1_a p8_f0_a p4_f1_a p4_f0_a p2_f1_a p2_f0_a p8_f1_b p8_f0_b p4_f1_b p4_f0_b p2_f1_b p2_f0_b ipc3_f1 ipc3_f0 h1 hdrv; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep -E 'passed|failed' gpurun_out/teng.log | tail -1; grep -E 'passed|failed' gpurun_out/ipc.log | tail -1
