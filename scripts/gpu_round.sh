#!/bin/bash
# One GPU-box session: tests, smoke, bench, profile. Each GPU step has its own time limit and the
# chain stops at the first failure (gpurun guidance: never retry a failing GPU step).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local t=$1; shift; echo "== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; return $rc; }
MODE=${1:-all}
export MDFX_SEGV_BACKTRACE=1
if [[ $MODE == all || $MODE == native ]]; then
  step 300 ./build/bin/mdfx_tests || exit 1
  step 300 ./build/bin/mdfx --stencil 7 --n 512 --steps 20 --warmup 5 --residual-every 10 || exit 1
fi
if [[ $MODE == all || $MODE == test ]]; then
  step 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
  tail -5 gpurun_out/pytest_gpu.log
fi
if [[ $MODE == all || $MODE == smoke ]]; then
  step 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step 300 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { cat gpurun_out/bench_n1.err; exit 1; }
  cat gpurun_out/bench_n1.json
  step 300 python bench.py --temporal 1 > gpurun_out/bench_n1_t1.json 2>> gpurun_out/bench_n1.err || exit 1
  cat gpurun_out/bench_n1_t1.json
  step 300 python bench.py --virtual-ranks 8 > gpurun_out/bench_v8.json 2>> gpurun_out/bench_n1.err || exit 1
  cat gpurun_out/bench_v8.json
fi
if [[ $MODE == all || $MODE == profile ]]; then
  R=$(pwd)
  (cd /tmp && export TMPDIR=/tmp && step 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python "$R/bench.py" --steps 20 --warmup 5 > "$R/gpurun_out/prof_bench.log" 2>&1) || { tail -20 gpurun_out/prof_bench.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
