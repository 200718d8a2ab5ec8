#!/bin/bash
# Round 3 session Q (re-entry after a container reset): the full GPU tier on the rebuilt tree, the
# native tests, ipc, smoke, the driver-style bench and one rocprof kernel-stats run.
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=600 scripts/gpu_session.sh native gputests ipc smoke || exit $?
scripts/gpu_session.sh "hdrv=python bench.py --steps 20 --warmup 5" "h1=python bench.py --steps 48 --warmup 12" || exit $?
PROF_TAG=q scripts/gpu_session.sh prof || exit $?
for f in hdrv h1; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep -E 'passed|failed' gpurun_out/gputests.log | tail -1
grep -E 'passed|failed' gpurun_out/ipc.log | tail -1
