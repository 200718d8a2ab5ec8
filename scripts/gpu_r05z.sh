#!/bin/bash
# Round 5, session Z: pencil candidates gated and timed at their own depth (4) next to the K = 5
# slabs: the 4-process headline-size ipc test, the proxy tests, and the 8-process rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipc.py \
  -k "headline_size or bench" tests/test_gpu_proxy.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $O/rehearsal8.json 2> $O/rehearsal8.err || { tail -20 $O/rehearsal8.err; exit 1; }
python - <<'PY'
import json
s = open("gpurun_out/r05z/rehearsal8.json").read()
r = json.loads(s[s.index('{"metric"'):].splitlines()[0])
c = r["config"]
print("rehearsal8", r["value"], c["transport"], c["temporal_block"], c["py"], c["verified"], c["repeats_ms_per_step"])
print("gate", [(g["transport"], g["graph"], g["py"], g["passed"]) for g in c["gate"]["runs"]])
PY
