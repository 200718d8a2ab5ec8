#!/bin/bash
# Round 3 session V: stream timeline of the N = 8 rank proxy (eager, the schedule the trials pick)
set -o pipefail
cd "$(dirname "$0")/.."
PROF_TAG=p8 BENCH_ARGS="--steps 48 --warmup 12 --rank-proxy 8 --graph off --rounds 1" scripts/gpu_session.sh prof || exit $?
PROF_TAG=p8ov0 BENCH_ARGS="--steps 48 --warmup 12 --rank-proxy 8 --graph off --rounds 1 --no-overlap" scripts/gpu_session.sh prof || exit $?
python3 scripts/kernel_timeline.py gpurun_out/prof_p8 --skip 200 > gpurun_out/timeline_p8.txt 2>&1
python3 scripts/kernel_timeline.py gpurun_out/prof_p8ov0 --skip 200 > gpurun_out/timeline_p8ov0.txt 2>&1
cat gpurun_out/timeline_p8.txt gpurun_out/timeline_p8ov0.txt
