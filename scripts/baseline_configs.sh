#!/bin/bash
# Every BASELINE.json config that fits one MI355X; JSON lines under gpurun_out/baseline_*.json.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local tag=$1; shift; echo "== $tag: $*"; timeout -k 10 600 python bench.py "$@" > gpurun_out/baseline_$tag.json 2> gpurun_out/baseline_$tag.err || { tail -5 gpurun_out/baseline_$tag.err; return 1; }; cat gpurun_out/baseline_$tag.json; }
run c2_heat7_512_f32 --n 512 --steps 100 --warmup 10 || exit 1
run c2_heat7_512_f32_t1 --n 512 --steps 100 --warmup 10 --temporal 1 || exit 1
run c3_heat7_1024_f32 --n 1024 --steps 50 --warmup 10 --repeats 2 || exit 1
run c4_box27_512_f32 --stencil box27 --n 512 --steps 100 --warmup 10 || exit 1
run c4_box27_512_f64 --stencil box27 --n 512 --dtype f64 --steps 50 --warmup 5 || exit 1
run c5_heat7_2048_f64_resid --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12 || exit 1
run c5_heat7_2048_f64_resid10 --n 2048 --dtype f64 --steps 20 --warmup 2 --residual-every 10 || exit 1
run x_heat7_1024_f64 --n 1024 --dtype f64 --steps 30 --warmup 5 || exit 1
run x_mdf2d_16k_f32 --stencil jacobi5 --nx 16384 --nz 16384 --steps 100 --warmup 10 || exit 1
run x_life_32k --stencil life --dtype u8 --nx 32768 --nz 32768 --steps 100 --warmup 10 || exit 1
run x_box27_1024_f32 --stencil box27 --n 1024 --steps 20 --warmup 4 || exit 1
run x_mdf2d_16k_f64 --stencil jacobi5 --dtype f64 --nx 16384 --nz 16384 --steps 100 --warmup 10 || exit 1
run x_heat7_1024_f32_v8 --n 1024 --steps 50 --warmup 10 --virtual-ranks 8 || exit 1
run x_heat7_1024_f32_ipc2 --n 1024 --steps 50 --warmup 10 --gpus 2 --share-gpu --transport ipc || exit 1
