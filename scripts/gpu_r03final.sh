#!/bin/bash
# Round 3, last session on the final tree: the full GPU tier (as the driver runs it), native, ipc,
# smoke, the driver-style bench and the MDF dialogue.
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=600 scripts/gpu_session.sh native gputests ipc smoke || exit $?
scripts/gpu_session.sh "drv=python bench.py --steps 20 --warmup 5" "dflt=python bench.py" "p8=python bench.py --steps 48 --warmup 12 --rank-proxy 8" || exit $?
printf '100\n16384\n16384\n' | timeout -k 10 120 ./build/bin/mdf --json > gpurun_out/final_dialogue.json 2>&1 || exit 1
for f in drv dflt p8; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
echo "dialogue $(grep -o '"value": [0-9.]*' gpurun_out/final_dialogue.json)"
grep -E 'passed|failed' gpurun_out/gputests.log | tail -1; grep -E 'passed|failed' gpurun_out/ipc.log | tail -1; tail -n 1 gpurun_out/native.log
