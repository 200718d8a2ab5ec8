#!/bin/bash
# Round 3 session S: warm_kernels (first launches outside the timed loop) in the CLI; the reference
# dialogue three times; then every BASELINE config on the current defaults (fp64 heat7_wxk 3+1 from
# 2048-cell rows).
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
scripts/gpu_session.sh "twarm=$PYT tests/test_gpu_engine.py -k 'warm' tests/test_gpu_cli.py" || exit $?
grep -q ' passed' gpurun_out/twarm.log && ! grep -q 'failed' gpurun_out/twarm.log || { tail -30 gpurun_out/twarm.log; exit 1; }
for i in 1 2 3; do
  printf '100\n16384\n16384\n' | timeout -k 10 120 ./build/bin/mdf --json > gpurun_out/dialogue_$i.json 2>&1 || exit 1
  echo "dialogue_$i $(grep -o '"value": [0-9.]*' gpurun_out/dialogue_$i.json)"
done
timeout -k 10 1000 bash scripts/baseline_configs.sh > gpurun_out/baseline.log 2>&1 || { tail -20 gpurun_out/baseline.log; exit 1; }
for f in gpurun_out/baseline_*.json; do echo "$(basename $f .json) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
