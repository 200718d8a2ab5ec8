#!/bin/bash
# Round 3 session W: window depth of the boundary-region launches only (MDFX_WXK_BNB) on the rank
# proxies (the boundary kernel of the N = 8 slab took 100 us of a 323 us sweep in session V)
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "tbnb=MDFX_WXK_BNB=31 $PYT tests/test_gpu_temporal.py -k 'wxk_regions_and_engine' tests/test_gpu_proxy.py" || exit $?
grep -q ' passed' gpurun_out/tbnb.log && ! grep -q 'failed' gpurun_out/tbnb.log || { tail -30 gpurun_out/tbnb.log; exit 1; }
P="python bench.py --steps 48 --warmup 12 --rank-proxy"
steps=()
for pass in a b; do
  for n in 8 4; do steps+=("p${n}_0_$pass=$P $n" "p${n}_31_$pass=MDFX_WXK_BNB=31 $P $n" "p${n}_32_$pass=MDFX_WXK_BNB=32 $P $n"); done
done
steps+=("p2_0=$P 2" "p2_31=MDFX_WXK_BNB=31 $P 2" "v8_0=python bench.py --steps 48 --warmup 12 --virtual-ranks 8" "v8_31=MDFX_WXK_BNB=31 python bench.py --steps 48 --warmup 12 --virtual-ranks 8")
scripts/gpu_session.sh "${steps[@]}" || exit $?
PROF_TAG=p8b31 BENCH_ARGS="--steps 48 --warmup 12 --rank-proxy 8 --graph off --rounds 1" MDFX_WXK_BNB=31 scripts/gpu_session.sh prof || exit $?
python3 scripts/kernel_timeline.py gpurun_out/prof_p8b31 --skip 200 > gpurun_out/timeline_p8b31.txt 2>&1
head -12 gpurun_out/timeline_p8b31.txt
for f in p8_0_a p8_31_a p8_32_a p4_0_a p4_31_a p4_32_a p8_0_b p8_31_b p8_32_b p4_0_b p4_31_b p4_32_b p2_0 p2_31 v8_0 v8_31; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
