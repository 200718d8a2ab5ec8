#!/bin/bash
# Round 5, session G3: every BASELINE config that fits one MI355X (scripts/baseline_configs.sh).
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=1000 scripts/gpu_session.sh "baseline=bash scripts/baseline_configs.sh" || exit $?
for f in gpurun_out/baseline_*.json; do echo "$(basename $f .json) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
