#!/bin/bash
# Round 4 session V: the final tree (sweep planner module, bounded watchdog reports): native tests,
# the whole GPU tier, smoke() and the driver's N = 1 bench forms.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh native || exit $?
tail -1 gpurun_out/native.log
LIMIT=900 scripts/gpu_session.sh "gputests=python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests" || exit $?
grep -E "passed|failed" gpurun_out/gputests.log | tail -2
scripts/gpu_session.sh smoke "b_default=python bench.py" "b_driver=python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
for f in b_default b_driver; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
