set -o pipefail
bash scripts/gpu_session.sh pmc_fetch pmc_write && \
PMC_TAG=f64_2048 BENCH_ARGS="--dtype f64 --n 2048 --residual-every 6 --graph off" bash scripts/gpu_session.sh pmc_fetch pmc_write && \
PMC_TAG=box27_f32 BENCH_ARGS="--stencil box27 --n 512 --graph off" bash scripts/gpu_session.sh pmc_fetch pmc_write && \
PMC_TAG=box27_f64 BENCH_ARGS="--stencil box27 --dtype f64 --n 512 --graph off" bash scripts/gpu_session.sh pmc_fetch pmc_write
