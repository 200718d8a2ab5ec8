#!/bin/bash
# Round 3 session AF: rocprofv3 kernel stats of the final tree: the headline bench and the fp64 / fp32 MDF 2D benches.
set -o pipefail
cd "$(dirname "$0")/.."
PROF_TAG=af_heat7 scripts/gpu_session.sh prof || exit $?
PROF_TAG=af_mdf64 BENCH_ARGS="--stencil jacobi5 --dtype f64 --nx 16384 --nz 16384 --steps 96 --warmup 16" scripts/gpu_session.sh prof || exit $?
PROF_TAG=af_mdf32 BENCH_ARGS="--stencil jacobi5 --nx 16384 --nz 16384 --steps 96 --warmup 16" scripts/gpu_session.sh prof || exit $?
ls -R gpurun_out/prof_af_* | head -30
