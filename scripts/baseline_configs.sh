#!/bin/bash
# Every BASELINE.json config that fits one MI355X (plus the reference's own MDF dialogue and the
# rank proxies of the N-GPU runs); JSON lines under gpurun_out/baseline_*.json.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
# (c5: the warm-up is a whole residual interval, so the timed window starts on a residual
# boundary; with --warmup 3 the window held a 4 + 4 + 1 and a 3-step stretch, profiles/r04_session_z/)
run() { local tag=$1; shift; echo "== $tag: $*"; timeout -k 10 600 python bench.py "$@" > gpurun_out/baseline_$tag.json 2> gpurun_out/baseline_$tag.err || { tail -5 gpurun_out/baseline_$tag.err; return 1; }; cat gpurun_out/baseline_$tag.json; }
run c1_mdf2d_256_f32_cpu --device cpu --stencil jacobi5 --nx 256 --nz 256 --steps 200 --warmup 10 || exit 1
run c2_heat7_512_f32 --n 512 --steps 100 --warmup 10 || exit 1
run c2_heat7_512_f32_t1 --n 512 --steps 100 --warmup 10 --temporal 1 || exit 1
run c3_heat7_1024_f32 --n 1024 --steps 50 --warmup 10 || exit 1
run c3_heat7_1024_f32_driver --n 1024 --steps 20 --warmup 5 || exit 1
for n in 2 4 8; do run c3_proxy$n --rank-proxy $n --steps 50 --warmup 10 || exit 1; done  # (K = 5: whole sweeps)
run c3_proxy8_pencil --rank-proxy 8 --py 2 --steps 48 --warmup 12 || exit 1
run c4_box27_512_f32 --stencil box27 --n 512 --steps 100 --warmup 10 || exit 1
run c4_box27_512_f64 --stencil box27 --n 512 --dtype f64 --steps 50 --warmup 5 || exit 1
run c5_heat7_2048_f64_resid --n 2048 --dtype f64 --steps 24 --warmup 12 --residual-every 12 || exit 1
run c5_heat7_2048_f64_resid10 --n 2048 --dtype f64 --steps 20 --warmup 10 --residual-every 10 || exit 1
run c5_heat7_2048_f64_resid20 --n 2048 --dtype f64 --steps 20 --warmup 20 --residual-every 20 || exit 1
run c5_proxy8_2048_f64_resid10 --rank-proxy 8 --n 2048 --dtype f64 --steps 20 --warmup 10 --residual-every 10 || exit 1
run c5_proxy8_2048_f64_resid --rank-proxy 8 --n 2048 --dtype f64 --steps 24 --warmup 12 --residual-every 12 || exit 1
run x_heat7_1024_f64 --n 1024 --dtype f64 --steps 30 --warmup 5 || exit 1
run x_mdf2d_16k_f32 --stencil jacobi5 --nx 16384 --nz 16384 --steps 96 --warmup 16 || exit 1
run x_mdf2d_16k_f32_ref --stencil jacobi5 --nx 16384 --nz 16384 --steps 96 --warmup 16 --ref-precision || exit 1
run x_mdf2d_16k_f64 --stencil jacobi5 --dtype f64 --nx 16384 --nz 16384 --steps 96 --warmup 16 || exit 1
run x_life_32k --stencil life --dtype u8 --nx 32768 --nz 32768 --steps 96 --warmup 12 || exit 1
run x_box27_1024_f32 --stencil box27 --n 1024 --steps 20 --warmup 4 || exit 1
run x_heat7_3072_f32 --n 3072 --steps 20 --warmup 5 || exit 1
run x_heat7_1024_f32_v8 --n 1024 --steps 50 --warmup 10 --virtual-ranks 8 || exit 1
run x_heat7_1024_f32_ipc2 --n 1024 --steps 50 --warmup 10 --gpus 2 --share-gpu --transport ipc || exit 1
echo "== mdf dialogue (reference-compatible CLI, reference precision, fused)"
printf '100\n16384\n16384\n' | timeout -k 10 300 ./build/bin/mdf --json > gpurun_out/baseline_mdf_dialogue.json 2>&1 || exit 1
tail -1 gpurun_out/baseline_mdf_dialogue.json
