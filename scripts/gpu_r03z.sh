#!/bin/bash
# Round 3 session Z (final tree, after the schedule changes): the full GPU tier, native tests, ipc, smoke, the driver-style
# bench twice, the default bench, the rank proxies, a rocprofv3 kernel-stats run and the FETCH /
# WRITE counter passes of the headline.
set -o pipefail
cd "$(dirname "$0")/.."
LIMIT=600 scripts/gpu_session.sh native gputests ipc smoke || exit $?
P="python bench.py --steps 48 --warmup 12 --rank-proxy"
scripts/gpu_session.sh "drv1=python bench.py --steps 20 --warmup 5" "dflt=python bench.py" "drv2=python bench.py --steps 20 --warmup 5" \
  "p2=$P 2" "p4=$P 4" "p8=$P 8" || exit $?
PROF_TAG=z scripts/gpu_session.sh prof || exit $?
PMC_TAG=z scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
for f in drv1 dflt drv2 p2 p4 p8; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
grep -E 'passed|failed' gpurun_out/gputests.log | tail -1
grep -E 'passed|failed' gpurun_out/ipc.log | tail -1
