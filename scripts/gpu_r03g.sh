#!/bin/bash
# Round 3 session G: heat7_wxk (y halo exchanged through LDS) -- bitwise tier, then A/B against
# heat7_wtk on the headline and the other heat7 configs.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --steps 48 --warmup 12"
scripts/gpu_session.sh "wxk=$PYT tests/test_gpu_temporal.py -k 'wxk'" || exit $?
grep -q ' passed' gpurun_out/wxk.log && ! grep -q 'failed' gpurun_out/wxk.log || { tail -30 gpurun_out/wxk.log; exit 1; }
W="MDFX_H7_WXK=1"
scripts/gpu_session.sh "wtk3=$B" "wxk3=$W $B" "wxk3r3=$W MDFX_WXK_RY=3 $B" "wxk4=$W $B --temporal 4" "wxk4r2=$W MDFX_WXK_RY=2 $B --temporal 4" \
  "wtk3_b=$B" "wxk3_b=$W $B" "wxk4_b=$W $B --temporal 4" "wxk3_drv=$W python bench.py --steps 20 --warmup 5" \
  "wxk4_drv=$W python bench.py --steps 20 --warmup 5 --temporal 4" \
  "wtk512=$B --n 512" "wxk512=$W $B --n 512" "wxk512k4=$W $B --n 512 --temporal 4" \
  "wtkp8=python bench.py --rank-proxy 8 --steps 48 --warmup 12" "wxkp8=$W python bench.py --rank-proxy 8 --steps 48 --warmup 12" \
  "wtk64=$B --dtype f64" "wxk64=$W $B --dtype f64" || exit $?
PMC_TAG=wxk3 MDFX_H7_WXK=1 scripts/gpu_session.sh pmc_fetch || exit $?
PMC_TAG=wxk4 MDFX_H7_WXK=1 BENCH_ARGS="--temporal 4" scripts/gpu_session.sh pmc_fetch || exit $?
for f in wtk3 wxk3 wxk3r3 wxk4 wxk4r2 wtk3_b wxk3_b wxk4_b wxk3_drv wxk4_drv wtk512 wxk512 wxk512k4 wtkp8 wxkp8 wtk64 wxk64; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
