#!/bin/bash
# heat7_wtk K = 3 against the default K = 2 kernels on the BASELINE shapes, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12 --graph on"
W="MDFX_H7_WTK=1"
steps=()
for rep in a b; do
  steps+=("c_1024_k2_$rep=$B --temporal 2" "c_1024_k3_$rep=$W $B --temporal 3"
          "c_512_k2_$rep=$B --n 512 --temporal 2" "c_512_k3_$rep=$W $B --n 512 --temporal 3"
          "c_1024f64_k2_$rep=$B --dtype f64 --temporal 2" "c_1024f64_k3_$rep=$W $B --dtype f64 --temporal 3"
          "c_v8_k2_$rep=$B --virtual-ranks 8 --temporal 2" "c_v8_k3_$rep=$W $B --virtual-ranks 8 --temporal 3")
done
LIMIT=300 scripts/gpu_session.sh "${steps[@]}" \
  "c_2048f64_k2=$B --n 2048 --dtype f64 --residual-every 10 --steps 30 --warmup 6 --temporal 2" \
  "c_2048f64_k3=$W $B --n 2048 --dtype f64 --residual-every 10 --steps 30 --warmup 6 --temporal 3" || exit $?
for f in gpurun_out/c_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
