#!/bin/bash
# Round 3 session L: heat7_wxk K = 4 band shapes 2+2 / 3+2 / 4+2 (inner + edge rows) across the
# headline, 512^3 and the rank proxies.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "wxk=$PYT tests/test_gpu_temporal.py -k 'wxk'" || exit $?
grep -q ' passed' gpurun_out/wxk.log && ! grep -q 'failed' gpurun_out/wxk.log || { tail -30 gpurun_out/wxk.log; exit 1; }
S="python bench.py --stencil box27 --steps 48 --warmup 12"
scripts/gpu_session.sh "b27k2=$S --n 512" "b27k3=$S --n 512 --temporal 3" "b27k2_b=$S --n 512" "b27k3_b=$S --n 512 --temporal 3" \
  "b27f64k2=$S --n 512 --dtype f64" "b27f64k3=$S --n 512 --dtype f64 --temporal 3" \
  "b27_1024k3=$S --n 1024 --temporal 3 --steps 24 --warmup 6" || exit $?
grep -q ' passed' gpurun_out/wxk.log && ! grep -q 'failed' gpurun_out/wxk.log || { tail -30 gpurun_out/wxk.log; exit 1; }
B="python bench.py --steps 48 --warmup 12"
P="python bench.py --steps 48 --warmup 12 --rank-proxy"
steps=()
for ry in 2 32 42; do steps+=("a$ry=MDFX_WXK_RY=$ry $B"); done
for ry in 2 32 42; do steps+=("b$ry=MDFX_WXK_RY=$ry $B"); done
for ry in 32 42; do steps+=("drv$ry=MDFX_WXK_RY=$ry python bench.py --steps 20 --warmup 5"); done
for ry in 31 32 42; do steps+=("n512_$ry=MDFX_WXK_RY=$ry $B --n 512"); done
for ry in 32 42; do steps+=("p8_$ry=MDFX_WXK_RY=$ry $P 8" "p4_$ry=MDFX_WXK_RY=$ry $P 4" "p2_$ry=MDFX_WXK_RY=$ry $P 2"); done
steps+=("n3072_42=MDFX_WXK_RY=42 python bench.py --n 3072 --steps 12 --warmup 4" "n2048_42=MDFX_WXK_RY=42 python bench.py --n 2048 --steps 24 --warmup 4")
scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in gpurun_out/b27*.log gpurun_out/{a,b}{2,32,42}.log gpurun_out/drv*.log gpurun_out/n512_*.log gpurun_out/p[248]_*.log gpurun_out/n3072_42.log gpurun_out/n2048_42.log; do echo "$(basename $f .log) $(grep -o '"value": [0-9.]*' $f)"; done
