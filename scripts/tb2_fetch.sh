#!/bin/bash
# tb2 z-chunk sweep: time (A/B harness) and FETCH_SIZE per variant.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out/tbf"
V="STEPS=2,TBRY=2;STEPS=2,TBRY=2,ZC=16;STEPS=2,TBRY=2,ZC=32;STEPS=2,TBRY=2,ZC=64;STEPS=2,TBRY=2,ZC=256;STEPS=2,TBRY=4,ZC=32;STEPS=2,TBRY=1,ZC=32"
timeout -k 10 400 python3 "$R/bench/kernel_ab.py" --n 1024 --iters 10 --rounds 3 --variants "$V" --json "$R/gpurun_out/tbf/ab.json" 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp
for v in "STEPS=2,TBRY=2" "STEPS=2,TBRY=2,ZC=16" "STEPS=2,TBRY=2,ZC=32" "STEPS=2,TBRY=4,ZC=32"; do
  tag=$(echo $v | tr ',=' '__')
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/gpurun_out/tbf/$tag" -o run -- python3 "$R/bench/kernel_ab.py" --n 1024 --iters 3 --rounds 1 --variants "$v" > "$R/gpurun_out/tbf/$tag.log" 2>&1 || { echo "pmc $v failed"; exit 1; }
done
