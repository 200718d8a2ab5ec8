#!/bin/bash
# Round 3 session D: full GPU tier after the kernel changes, heat7_wtk z-chunk sweep (fetch
# counters), then every BASELINE config.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --steps 48 --warmup 12"
steps=("temporal=$PYT tests/test_gpu_temporal.py")
for zc in 0 74 98 128 205; do steps+=("zc$zc=MDFX_ZC=$zc $B"); done
steps+=("zc0_b=$B")
LIMIT=400 scripts/gpu_session.sh "${steps[@]}" || exit $?
PMC_TAG=zc74 BENCH_ARGS="" MDFX_ZC=74 scripts/gpu_session.sh pmc_fetch || exit $?
PMC_TAG=zc205 BENCH_ARGS="" MDFX_ZC=205 scripts/gpu_session.sh pmc_fetch || exit $?
LIMIT=1100 scripts/gpu_session.sh gputests || exit $?
timeout -k 10 1500 bash scripts/baseline_configs.sh > gpurun_out/baseline.log 2>&1 || { tail -20 gpurun_out/baseline.log; exit 1; }
for f in gpurun_out/zc*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
grep -h -o '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/baseline_*.json
tail -n 1 gpurun_out/baseline_mdf_dialogue.json
