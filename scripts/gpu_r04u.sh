#!/bin/bash
# Round 4 session U: the whole GPU tier, smoke(), the driver's default bench and N = 1 form, every
# BASELINE config and the 8-process shared-GPU rehearsal of the N = 8 bench, after the halo-priority change.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh native || exit $?
tail -2 gpurun_out/native.log
LIMIT=900 scripts/gpu_session.sh "gputests=python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests" || exit $?
grep -E "passed|failed" gpurun_out/gputests.log | tail -2
scripts/gpu_session.sh smoke "b_default=python bench.py" "b_driver=python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
for f in b_default b_driver; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
LIMIT=700 scripts/gpu_session.sh "baseline=bash scripts/baseline_configs.sh" || exit $?
for f in gpurun_out/baseline_*.json; do echo "$(basename $f .json) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
timeout -k 10 900 python bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > gpurun_out/rehearsal8.json 2> gpurun_out/rehearsal8.err || { tail -20 gpurun_out/rehearsal8.err; exit 1; }
grep -o '"value": [0-9.]*\|"transport": "[a-z_]*"\|"timed_vs_trial": [0-9.]*' gpurun_out/rehearsal8.json | head -4
