#!/bin/bash
# Kernel A/B sweeps for every family on one MI355X (bench/kernel_ab.py); logs under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ab() { local tag=$1; shift; echo "== $tag"; timeout -k 10 300 python bench/kernel_ab.py --json gpurun_out/ab_$tag.json "$@" > gpurun_out/ab_$tag.log 2>&1; local rc=$?; cat gpurun_out/ab_$tag.log | grep -v amdgpu.ids; return $rc; }
ab heat7_f64 --kind heat7 --dtype f64 --n 1024 --iters 10 --variants "FAM=naive;RY=2,PF=1;RY=2,PF=2;RY=4,PF=1;RY=4,PF=2;RY=1,PF=2" || exit 1
ab box27_f32 --kind box27 --n 512 --iters 20 --variants "FAM=naive;RY=1;RY=2;RY=4" || exit 1
ab box27_f64 --kind box27 --dtype f64 --n 512 --iters 10 --variants "FAM=naive;RY=1;RY=2" || exit 1
ab heat7_f32_512 --kind heat7 --n 512 --iters 40 --variants "RY=2,PF=1;RY=4,PF=1;RY=2,PF=1,BLOCKS=4096;RY=1,PF=1" || exit 1
ab jacobi5_f32 --kind jacobi5 --nx 16384 --nz 16384 --iters 20 --variants "FAM=naive;ZC=64;ZC=128;ZC=256;ZC=32" || exit 1
ab life_u8 --kind life --nx 32768 --nz 32768 --iters 20 --variants "FAM=naive;ZC=64;ZC=128;ZC=256" || exit 1
