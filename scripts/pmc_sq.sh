#!/bin/bash
# SQ counter pass (one rocprofv3 --pmc run, 8 SQ counters) over bench.py with $BENCH_ARGS;
# output gpurun_out/sq_$TAG. Usage: TAG=k3 BENCH_ARGS="--temporal 3" bash scripts/pmc_sq.sh
# (CTRS replaces the counter list: at most 8 SQ counters per pass)
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc ${CTRS:-SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
   SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY} --kernel-trace --output-format csv \
   -d "$R/gpurun_out/sq_$TAG" -o run -- python3 "$R/bench.py" --steps 12 --warmup 2 --graph off ${BENCH_ARGS:-} \
   > "$R/gpurun_out/sq_$TAG.log" 2>&1)
rc=$?; echo "== sq_$TAG rc=$rc"; tail -1 "$R/gpurun_out/sq_$TAG.log" | cut -c1-200; exit $rc
