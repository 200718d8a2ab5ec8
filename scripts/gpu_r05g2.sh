#!/bin/bash
# Round 5, session G2: the driver's bench forms, a kernel trace of the driver form, the 8-process
# shared-GPU rehearsal of the N = 8 bench (timed run verified).
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh "b_default=python bench.py" "b_driver=python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
for f in b_default b_driver; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
PROF_TAG=driver BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" scripts/gpu_session.sh prof || exit $?
timeout -k 10 600 python bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > gpurun_out/rehearsal8.json 2> gpurun_out/rehearsal8.err || { tail -20 gpurun_out/rehearsal8.err; exit 1; }
grep -o '"value": [0-9.]*\|"transport": "[a-z_]*"\|"verified": {[^}]*}\|"repeats_ms_per_step": \[[^]]*\]' gpurun_out/rehearsal8.json | head -5
