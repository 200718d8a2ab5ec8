#!/bin/bash
# A/B on one box: the headline bench of this tree against the session-Q tree (ecb205f, built in
# build/ab_q), interleaved, driver-style and 48-step runs.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
run() { local tag=$1 dir=$2; shift 2; (cd "$dir" && timeout -k 10 300 python bench.py "$@") > "$R/gpurun_out/abq_$tag.log" 2>&1 || { tail -5 "$R/gpurun_out/abq_$tag.log"; exit 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $R/gpurun_out/abq_$tag.log)"; }
for i in 1 2 3; do
  run head_drv_$i "$R" --steps 20 --warmup 5
  run q_drv_$i "$R/build/ab_q" --steps 20 --warmup 5
  run head_48_$i "$R" --steps 48 --warmup 12
  run q_48_$i "$R/build/ab_q" --steps 48 --warmup 12
done
