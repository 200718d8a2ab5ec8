#!/bin/bash
# Round 5, session AN: the final tree (split ghost waits): the driver's GPU-tier form, smoke
# and the driver form, on the final tree (K = 5, ghost events, IPC export retry).
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh native || exit $?
LIMIT=1150 scripts/gpu_session.sh "gputier=python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread" || exit $?
grep -E "passed|failed" gpurun_out/gputier.log | tail -2
grep -h "retries" gpurun_out/gputier.log gpurun_out/ipc_churn_stderr.log 2>/dev/null | head -3
scripts/gpu_session.sh smoke "b_driver=python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
echo "b_driver $(grep -o '"value": [0-9.]*' gpurun_out/b_driver.log)"
