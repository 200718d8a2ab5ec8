#!/bin/bash
# Round 3 session B: heat7_wtk row layouts (MDFX_WTK_NAT 0 / 1 / 2) bitwise + A/B, then the new
# engine / bootstrap tests, smoke, driver-style bench and the full GPU tier.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --steps 48 --warmup 12"
steps=("temporal=$PYT tests/test_gpu_temporal.py"
       "temporal_nat1=MDFX_WTK_NAT=1 $PYT tests/test_gpu_temporal.py -k wtk")
for r in a b; do
  for m in 0 1 2; do steps+=("h1024_nat${m}_$r=MDFX_WTK_NAT=$m $B"); done
done
for m in 0 1 2; do steps+=("v8_nat$m=MDFX_WTK_NAT=$m $B --virtual-ranks 8"); done
steps+=("newtests=$PYT -v tests/test_gpu_engine.py -k prepared tests/test_gpu_multiprocess.py -k bootstrap"
        smoke "drv=python bench.py --steps 20 --warmup 5" "dflt=python bench.py" gputests ipc)
LIMIT=600 scripts/gpu_session.sh "${steps[@]}" || exit $?
for f in gpurun_out/h1024_nat*.log gpurun_out/v8_nat*.log gpurun_out/drv.log gpurun_out/dflt.log; do
  echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"graph": [a-z]*, "graph_requested": [a-z]*, "graph_replays_timed": [0-9]*, "graph_captures_timed": [0-9]*' $f)"; done
tail -3 gpurun_out/gputests.log gpurun_out/ipc.log
