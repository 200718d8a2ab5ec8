#!/bin/bash
# Round 5, session X: the whole GPU tier, smoke() and the driver form with K = 5 as the default,
# plus a kernel trace and FETCH / WRITE passes of the driver form.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh native || exit $?
LIMIT=1100 scripts/gpu_session.sh "gputests=python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_ipc.py" || exit $?
grep -E "passed|failed" gpurun_out/gputests.log | tail -2
scripts/gpu_session.sh ipc smoke || exit $?
grep -E "passed|failed" gpurun_out/ipc.log | tail -1
scripts/gpu_session.sh "b_driver=python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
echo "b_driver $(grep -o '"value": [0-9.]*' gpurun_out/b_driver.log)"
PROF_TAG=k5 scripts/gpu_session.sh prof || exit $?
PMC_TAG=k5 scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
