#!/bin/bash
# Round 3 session AI: the proxy's timed run with graph replay trails its own trial 2-3x (K = 2 / K = 1 at N = 8):
# is it the init() before the timed run? graph on only, with and without it.
set -o pipefail
cd "$(dirname "$0")/.."
P="python bench.py --steps 48 --warmup 12 --rank-proxy 8 --temporal 2 --graph on --rounds 2"
scripts/gpu_session.sh "gi1=$P" "gi0=MDFX_PROXY_FINAL_INIT=0 $P" "ge=python bench.py --steps 48 --warmup 12 --rank-proxy 8 --temporal 2 --graph off --rounds 2" || exit $?
for f in gi1 gi0 ge; do echo "$f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/$f.log | tr '\n' ' ')"; done
