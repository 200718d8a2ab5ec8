#!/bin/bash
# Round 3 session N: which band shape the default 1024^3 run launches, against the forced shapes.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12"
scripts/gpu_session.sh "dbg=MDFX_DEBUG_ZC=1 python bench.py --steps 8 --warmup 4" "d1=$B" "r42=MDFX_WXK_RY=42 $B" "r32=MDFX_WXK_RY=32 $B" "d2=$B" "r42b=MDFX_WXK_RY=42 $B" || exit $?
grep -h 'wxk' gpurun_out/dbg.log | sort | uniq -c | head -20
for f in d1 r42 r32 d2 r42b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
