#!/bin/bash
# heat7_wtk 32- vs 64-lane x segments (fp32): bitwise tests, then 1024^3 / 512^3 / 2048^3 and the
# single-slab shapes of the 2 / 8-GPU runs.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on --temporal 3"
LIMIT=300 scripts/gpu_session.sh \
  "wtk_tests=python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -k wtk" \
  "hl_1024_64=MDFX_WTK_HL=64 $B" "hl_1024_32=MDFX_WTK_HL=32 $B" \
  "hl_512_64=MDFX_WTK_HL=64 $B --n 512" "hl_512_32=MDFX_WTK_HL=32 $B --n 512" "hl_512_k2=python bench.py --steps 48 --warmup 12 --graph on --n 512 --temporal 2" \
  "hl_2048_64=MDFX_WTK_HL=64 $B --n 2048 --steps 24 --warmup 6" "hl_2048_32=MDFX_WTK_HL=32 $B --n 2048 --steps 24 --warmup 6" \
  "hl_nz128_64=MDFX_WTK_HL=64 $B --nx 1024 --ny 1024 --nz 128" "hl_nz128_32=MDFX_WTK_HL=32 $B --nx 1024 --ny 1024 --nz 128" \
  "hl_1024_64b=MDFX_WTK_HL=64 $B" "hl_1024_32b=MDFX_WTK_HL=32 $B" || exit $?
for f in gpurun_out/hl_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
