#!/bin/bash
# Per-GPU slab shapes of the strong-scaling headline (1024 x 1024 x 1024/N): which kernel
# configuration is fastest when each GPU holds 512 / 256 / 128 planes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V="RY=2,PF=1;RY=2,PF=1,BLOCKS=2048;RY=2,PF=1,BLOCKS=8192;RY=4,PF=1;STEPS=2,TBRY=2,TBPF=1;STEPS=2,TBRY=2,TBPF=1,BLOCKS=2048;STEPS=2,TBRY=2,TBPF=1,BLOCKS=1024;STEPS=2,TBRY=1,TBPF=1;STEPS=2,TBRY=2,TBPF=0"
for nz in 512 256 128; do
  echo "== nz=$nz"
  timeout -k 10 300 python bench/kernel_ab.py --nx 1024 --ny 1024 --nz $nz --iters 30 --rounds 3 --variants "$V" --json gpurun_out/ab_slab_nz$nz.json 2>&1 | grep -v amdgpu.ids || exit 1
done
