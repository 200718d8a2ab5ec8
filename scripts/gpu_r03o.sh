#!/bin/bash
# Round 3 session O: defaults after sessions L-N (heat7_wxk 3+2 band at K = 4, box27_wxk K = 3 for
# fp64 / wide rows), fp64 heat7_wxk K = 3 against heat7_wtk, then every BASELINE config.
set -o pipefail
cd "$(dirname "$0")/.."
B="python bench.py --steps 48 --warmup 12"
scripts/gpu_session.sh "f64wtk=$B --dtype f64" "f64wxk=MDFX_H7_WXK=1 $B --dtype f64" \
  "f64rwtk=python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12" \
  "f64rwxk=MDFX_H7_WXK=1 python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12" || exit $?
timeout -k 10 1500 bash scripts/baseline_configs.sh > gpurun_out/baseline.log 2>&1 || { tail -20 gpurun_out/baseline.log; exit 1; }
for f in f64wtk f64wxk f64rwtk f64rwxk; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
for f in gpurun_out/baseline_*.json; do echo "$(basename $f .json) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
