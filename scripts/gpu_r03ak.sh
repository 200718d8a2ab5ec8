#!/bin/bash
# Round 3 session AK: is the slow graph replay in the N = 8 proxy tied to the buffer parity the timed run starts on?
# K = 2, graphs on: warm-up 12 steps (6 sweeps: timed run starts on parity 0) vs 14 (7 sweeps: parity 1).
set -o pipefail
cd "$(dirname "$0")/.."
P="python bench.py --steps 48 --rank-proxy 8 --temporal 2 --graph on --rounds 2"
scripts/gpu_session.sh "ak_w12=$P --warmup 12" "ak_w14=$P --warmup 14" "ak_w10=$P --warmup 10" "ak_w6=$P --warmup 6" || exit $?
for f in ak_w12 ak_w14 ak_w10 ak_w6; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
