#!/bin/bash
# Round 3 session A: new GPU tests (prepared graphs, bounded RCCL bootstrap), full GPU tier, smoke,
# driver-style and default bench.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
LIMIT=600 scripts/gpu_session.sh \
  "newtests=$PYT tests/test_gpu_engine.py -k prepared tests/test_gpu_multiprocess.py -k bootstrap" \
  smoke \
  "drv=python bench.py --steps 20 --warmup 5" \
  "dflt=python bench.py" \
  "drv2=python bench.py --steps 20 --warmup 5" \
  gputests ipc || exit $?
grep -h '"value"' gpurun_out/drv.log gpurun_out/dflt.log gpurun_out/drv2.log | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); c=r['config']; print(r['value'], r['steps'], r['warmup'], c['graph'], c['graph_replays_timed'], c['graph_captures_timed'])"
tail -3 gpurun_out/gputests.log gpurun_out/ipc.log
