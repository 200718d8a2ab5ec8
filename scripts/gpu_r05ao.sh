#!/bin/bash
# Round 5, session AO: longer verified multi-process runs on the final tree (processes sharing one
# GPU over ipc, K = 5 slabs / K = 4 pencils in the trials): 4 processes x 100 steps, 8 x 50.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ao
mkdir -p $O
for spec in "4 100 10" "8 50 10"; do
  set -- $spec
  timeout -k 10 900 python bench.py --gpus $1 --share-gpu --steps $2 --warmup $3 > $O/g$1.json 2> $O/g$1.err || { tail -20 $O/g$1.err; exit 1; }
  python - "$O/g$1.json" <<'PY'
import json, sys
s = open(sys.argv[1]).read()
r = json.loads(s[s.index('{"metric"'):].splitlines()[0])
c = r["config"]
print("gpus", r["n_gpus"], "steps", r["steps"], c["transport"], "py", c["py"], "K", c["temporal_block"], "verified", c["verified"]["passed"],
      c["verified"]["max_abs_diff"], "gate", all(g["passed"] for g in c["gate"]["runs"] if g["transport"] != "rccl"))
PY
done
