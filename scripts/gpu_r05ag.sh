#!/bin/bash
# Round 5, session AG: the whole GPU tier on the final tree (K = 5 default, ghost events), smoke,
# the driver form twice, and the 8-process shared-GPU rehearsal of the N = 8 command.
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh native || exit $?
LIMIT=1100 scripts/gpu_session.sh "gputests=python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_ipc.py" || exit $?
grep -E "passed|failed" gpurun_out/gputests.log | tail -2
scripts/gpu_session.sh ipc smoke || exit $?
grep -E "passed|failed" gpurun_out/ipc.log | tail -1
scripts/gpu_session.sh "b_driver=python bench.py --gpus 1 --steps 20 --warmup 5" "b_driver2=python bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
for f in b_driver b_driver2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
timeout -k 10 600 python bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > gpurun_out/rehearsal8.json 2> gpurun_out/rehearsal8.err || { tail -20 gpurun_out/rehearsal8.err; exit 1; }
grep -o '"verified": {[^}]*}\|"temporal_block": [0-9]*\|"transport": "[a-z_]*"' gpurun_out/rehearsal8.json | tail -3
