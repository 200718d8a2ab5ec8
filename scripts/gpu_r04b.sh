#!/bin/bash
# Round 4 session B: heat7_wxk L2 prefetch of plane q + 2 (MDFX_WXK_PF byte strides) bitwise and
# timed; the pruned wxk instances; ipc / proxy protocols x copy engines with concurrent pulls.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "wxk_t=$PYT tests/test_gpu_temporal.py -k wxk" "proxy_t=$PYT tests/test_gpu_proxy.py" \
  "ipc_t=$PYT tests/test_gpu_ipc.py" || exit $?
B="python bench.py --steps 20 --warmup 5"
scripts/gpu_session.sh "pf0=MDFX_WXK_PF=0 $B" "pf64=MDFX_WXK_PF=64 $B" "pf128=MDFX_WXK_PF=128 $B" "pf256=MDFX_WXK_PF=256 $B" \
  "pf0b=MDFX_WXK_PF=0 $B" "pf64b=MDFX_WXK_PF=64 $B" "pf128b=MDFX_WXK_PF=128 $B" \
  "p8=python bench.py --rank-proxy 8 --steps 48 --warmup 5" "p8pf=MDFX_WXK_PF=128 python bench.py --rank-proxy 8 --steps 48 --warmup 5" \
  "p4=python bench.py --rank-proxy 4 --steps 48 --warmup 5" || exit $?
for f in pf0 pf64 pf128 pf256 pf0b pf64b pf128b p8 p8pf p4; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"timed_vs_trial": [0-9.a-z]*' gpurun_out/$f.log)"; done
