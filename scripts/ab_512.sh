#!/bin/bash
set -o pipefail
cd /root/repo
B="python bench.py --steps 48 --warmup 12 --graph on --n 512"
LIMIT=300 scripts/gpu_session.sh "t512_k2=$B --temporal 2" "t512_tbk3=MDFX_H7_WTK=-1 $B --temporal 3" \
  "t512_tbk3r1=MDFX_H7_WTK=-1 MDFX_TBK_RY=1 $B --temporal 3" "t512_tbk4=MDFX_H7_WTK=-1 $B --temporal 4" \
  "t512_k2r2=MDFX_TBK_RY=2 $B --temporal 2" "t512_k2b=$B --temporal 2" || exit $?
for f in gpurun_out/t512_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
