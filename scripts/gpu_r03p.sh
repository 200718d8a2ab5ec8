#!/bin/bash
# Round 3 session P: boundary-first schedule on the rank proxies / multi-slab runs, fp64 heat7_wxk
# band shapes against heat7_wtk.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "wxk=$PYT tests/test_gpu_temporal.py -k 'wxk' tests/test_gpu_engine.py tests/test_gpu_proxy.py" "fallback=$PYT tests/test_gpu_multiprocess.py -k 'fallback or bootstrap'" || exit $?
grep -q ' passed' gpurun_out/fallback.log && ! grep -q 'failed' gpurun_out/fallback.log || { tail -30 gpurun_out/fallback.log; exit 1; }
grep -q ' passed' gpurun_out/wxk.log && ! grep -q 'failed' gpurun_out/wxk.log || { tail -30 gpurun_out/wxk.log; exit 1; }
B="python bench.py --steps 48 --warmup 12"
P="python bench.py --steps 48 --warmup 12 --rank-proxy"
steps=()
for bf in 1 0; do steps+=("p8_bf$bf=MDFX_BND_FIRST=$bf $P 8" "p4_bf$bf=MDFX_BND_FIRST=$bf $P 4" "p2_bf$bf=MDFX_BND_FIRST=$bf $P 2" "v8_bf$bf=MDFX_BND_FIRST=$bf $B --virtual-ranks 8"); done
steps+=("p8_bf1b=MDFX_BND_FIRST=1 $P 8" "p8_bf0b=MDFX_BND_FIRST=0 $P 8" "ipc2=$B --gpus 2 --share-gpu --transport ipc")
steps+=("f64wtk=$B --dtype f64" "f64x22=MDFX_H7_WXK=1 $B --dtype f64" "f64x32=MDFX_H7_WXK=1 MDFX_WXK_RY=32 $B --dtype f64" "f64x31=MDFX_H7_WXK=1 MDFX_WXK_RY=31 $B --dtype f64")
R="python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12"
steps+=("r_wtk=$R" "r_x22=MDFX_H7_WXK=1 $R" "r_x32=MDFX_H7_WXK=1 MDFX_WXK_RY=32 $R" "r_x31=MDFX_H7_WXK=1 MDFX_WXK_RY=31 $R")
scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in p8_bf1 p4_bf1 p2_bf1 v8_bf1 p8_bf0 p4_bf0 p2_bf0 v8_bf0 p8_bf1b p8_bf0b ipc2 f64wtk f64x22 f64x32 f64x31 r_wtk r_x22 r_x32 r_x31; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
