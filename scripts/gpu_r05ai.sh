#!/bin/bash
# Round 5, session AI: every BASELINE config on the final tree (K = 5 default, ghost events).
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=1100 scripts/gpu_session.sh "baseline=bash scripts/baseline_configs.sh" || exit $?
for f in gpurun_out/baseline_*.json; do echo "$(basename $f .json) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
