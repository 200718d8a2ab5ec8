#!/bin/bash
# Interleaved A/B (bench/kernel_ab.py: variants alternate in ONE process, best / median of rounds)
# for the fused 27-point kernels and the 7-point tile height; logs under gpurun_out/abi_*.log.
set -o pipefail
cd "$(dirname "$0")/.."
A="timeout -k 10 300 python bench/kernel_ab.py --rounds 5"
$A --kind box27 --n 512 --dtype f32 --iters 20 --variants "STEPS=2,B27TBK=-1;STEPS=2,B27TBK=2;STEPS=2,B27TBK=4" > gpurun_out/abi_b27_512_f32.log 2>&1 || exit 1
$A --kind box27 --n 1024 --dtype f32 --iters 6 --variants "STEPS=2,B27TBK=-1;STEPS=2,B27TBK=2;STEPS=2,B27TBK=4" > gpurun_out/abi_b27_1024_f32.log 2>&1 || exit 1
$A --kind box27 --n 512 --dtype f64 --iters 20 --variants "STEPS=2,B27TBK=-1;STEPS=2,B27TBK=2;STEPS=2,B27TBK=4" > gpurun_out/abi_b27_512_f64.log 2>&1 || exit 1
$A --kind heat7 --n 1024 --dtype f32 --iters 10 --variants "STEPS=2,TBKRY=4;STEPS=2,TBKRY=2;STEPS=3,TBKRY=2;STEPS=2,TBKRY=1" > gpurun_out/abi_h7_1024.log 2>&1 || exit 1
$A --kind heat7 --nx 1024 --ny 1024 --nz 128 --dtype f32 --iters 20 --variants "STEPS=2,TBKRY=4;STEPS=2,TBKRY=2;STEPS=2,TBKRY=4,ZC=32;STEPS=2,TBKRY=4,ZC=128" > gpurun_out/abi_h7_slab.log 2>&1 || exit 1
