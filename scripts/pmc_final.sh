#!/bin/bash
# Counter passes of the shipped 1024^3 fp32 K = 3 sweep (heat7_wtk): FETCH_SIZE, WRITE_SIZE, SQ.
set -o pipefail
cd "$(dirname "$0")/.."
PMC_TAG=final BENCH_ARGS="--temporal 3" scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
TAG=final BENCH_ARGS="--temporal 3" bash scripts/pmc_sq.sh || exit $?
python3 scripts/pmc_sq_summary.py gpurun_out/sq_final > gpurun_out/sq_summary_final.txt
python3 scripts/pmc_bytes.py gpurun_out final --field-bytes 4294967296 > gpurun_out/pmc_bytes_final.txt
