#!/bin/bash
# Round 3 session AE: why is the timed run 2-5% slower than the best trial of the same process?
# Warm-up length (grid state / clocks after init) vs timed length, same tree.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh "w5=python bench.py --steps 20 --warmup 5" "w100=python bench.py --steps 20 --warmup 100" \
  "w400=python bench.py --steps 20 --warmup 400" "s200=python bench.py --steps 200 --warmup 5" \
  "w5b=python bench.py --steps 20 --warmup 5 --repeats 5" || exit $?
for f in w5 w100 w400 s200 w5b; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1) trials $(grep -o '"trials": \[[^]]*' gpurun_out/$f.log | grep -o 'ms_per_step": [0-9.]*' | tr '\n' ' ')"; done
