#!/bin/bash
# Round 5, session I: the ipc multi-process tests with the graph runs asserted to replay and the
# captured graphs checked for fold waits.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh ipc || exit $?
grep -E "passed|failed" gpurun_out/ipc.log | tail -1
