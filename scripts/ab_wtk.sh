#!/bin/bash
# heat7_wtk A/B on one GPU: bitwise tests, then bench.py at 1024^3 fp32 for the shipped
# heat7_tbk and heat7_wtk variants (MDFX_WTK_RY rows per wave, MDFX_WTK_NB u0 planes in flight,
# MDFX_WTK_ORDER task order, MDFX_ZC z chunk), then a FETCH_SIZE pass of the default wtk.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
W="MDFX_H7_WTK=1"
LIMIT=300 scripts/gpu_session.sh \
  "wtk_tests=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -k wtk" \
  "ab_tbk2=$B --temporal 2" \
  "ab_wtk3_o1=$W MDFX_WTK_ORDER=1 $B --temporal 3" \
  "ab_wtk3_o0=$W $B --temporal 3" \
  "ab_wtk3_o0_zc64=$W MDFX_ZC=64 $B --temporal 3" \
  "ab_wtk3_o0_zc128=$W MDFX_ZC=128 $B --temporal 3" \
  "ab_wtk3_o0_r2=$W MDFX_WTK_RY=2 $B --temporal 3" \
  "ab_wtk2_o0_r4=$W $B --temporal 2" \
  "ab_wtk4_o0=$W $B --temporal 4" \
  "ab_wtk3_o0b=$W $B --temporal 3" \
  "ab_tbk2b=$B --temporal 2" || exit $?
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
MDFX_H7_WTK=1 PMC_TAG=wtk3o0 BENCH_ARGS="--temporal 3" scripts/gpu_session.sh pmc_fetch
