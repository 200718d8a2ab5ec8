#!/bin/bash
# Round 3 session T: box27_wxp (27-point K = 3 in two 256-cell x halves per block, rows 257..512)
# bitwise tier, then 512^3 fp32 against box27_tb2n (K = 2) and the overlapping-segment box27_wxk.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "tb27=$PYT tests/test_gpu_temporal.py -k 'box27' tests/test_gpu_engine.py -k 'box27 or warm or auto'" || exit $?
grep -q ' passed' gpurun_out/tb27.log && ! grep -q 'failed' gpurun_out/tb27.log || { tail -40 gpurun_out/tb27.log; exit 1; }
B="python bench.py --stencil box27 --n 512 --steps 48 --warmup 12"
steps=()
for pass in a b; do
  steps+=("xp_$pass=$B" "tb2n_$pass=MDFX_B27_WXK=0 $B" "wxk_$pass=MDFX_B27_WXP=0 MDFX_B27_WXK=1 $B")
done
steps+=("xp_c4=python bench.py --stencil box27 --n 512 --steps 100 --warmup 10" "xp_p8=python bench.py --stencil box27 --n 512 --steps 48 --warmup 12 --rank-proxy 8")
scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in xp_a tb2n_a wxk_a xp_b tb2n_b wxk_b xp_c4 xp_p8; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
