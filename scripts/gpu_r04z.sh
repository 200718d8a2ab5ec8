#!/bin/bash
# Round 4, session Z: rocprofv3 kernel statistics of the final tree's headline bench (driver form)
# and of the fp64 residual config (c5), for the bench <-> profiler cross-check.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out/zz"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/zz/headline" -o run -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$R/gpurun_out/zz/headline.log" 2>&1 || { tail -20 "$R/gpurun_out/zz/headline.log"; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$R/gpurun_out/zz/headline.log" | head -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/zz/c5" -o run -- \
  python3 "$R/bench.py" --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12 > "$R/gpurun_out/zz/c5.log" 2>&1 || { tail -20 "$R/gpurun_out/zz/c5.log"; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' "$R/gpurun_out/zz/c5.log" | head -2
