#!/bin/bash
# Round 5, session AP: after the last library change (an error message): the ipc tests and smoke.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh ipc smoke || exit $?
grep -E "passed|failed" gpurun_out/ipc.log | tail -1
