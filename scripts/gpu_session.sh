#!/bin/bash
# One GPU-box session of named steps. Each step runs under its own time limit and logs to
# gpurun_out/<name>.log. A step that merely fails (exit 1: a failed assertion) lets the next one
# run; a crash, abort, signal or time limit (any other non-zero status) ends the session there
# (gpurun rules: no further GPU work after a fault, no retries).
#
#   scripts/gpu_session.sh <step> [<step> ...]     steps: native ipc gputests smoke bench bench_t1
#                                                  bench_v8 prof pmc_fetch pmc_write, or name=command
#                                                  (limit $LIMIT s, default 300)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$(pwd)
PYT="python -u -m pytest -v --timeout 120 --timeout-method thread"

run() {  # run <limit_s> <name> cmd...
  local t=$1 name=$2
  shift 2
  echo "== $(date +%T) $name (limit ${t}s): $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then
    echo "== stopping: $name ended with status $rc"
    exit $rc
  fi
  return 0
}

for s in "$@"; do
  case $s in
    native) run 300 native ./build/bin/mdfx_tests ;;
    ipc) run 600 ipc $PYT tests/test_gpu_ipc.py ;;
    gputests) run 1100 gputests $PYT -m gpu tests --deselect tests/test_gpu_ipc.py ;;
    smoke) run 300 smoke python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 300 bench python bench.py ;;
    bench_t1) run 300 bench_t1 python bench.py --temporal 1 ;;
    bench_v8) run 300 bench_v8 python bench.py --virtual-ranks 8 ;;
    bench_ipc2) run 300 bench_ipc2 python bench.py --gpus 2 --share-gpu --transport ipc ;;
    bench_ipc4) run 300 bench_ipc4 python bench.py --gpus 4 --share-gpu --transport ipc ;;
    bench_refuse) run 120 bench_refuse bash -c 'python bench.py --gpus 2 --n 256; test $? -eq 2' ;;  # must refuse
    rccl2) run 150 rccl2 python bench.py --gpus 2 --share-gpu --transport rccl --n 256 --steps 4 --warmup 2 ;;
    prof)  # kernel trace + stats of one bench run (PROF_TAG names it, BENCH_ARGS replaces the bench flags)
      out="prof${PROF_TAG:+_$PROF_TAG}"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
          --output-format csv -d "$R/gpurun_out/$out" -o bench -- python3 "$R/bench.py" ${BENCH_ARGS:---steps 20 --warmup 5} \
          > "$R/gpurun_out/$out.log" 2>&1); rc=$?; echo "== $out rc=$rc"; tail -2 "gpurun_out/$out.log"; [[ $rc -le 1 ]] || exit $rc ;;
    pmc_fetch|pmc_write)  # one counter per pass (FETCH_SIZE and WRITE_SIZE cannot share one)
      ctr=$([[ $s == pmc_fetch ]] && echo FETCH_SIZE || echo WRITE_SIZE)
      out="$s${PMC_TAG:+_$PMC_TAG}"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
          -d "$R/gpurun_out/$out" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 ${BENCH_ARGS:-} \
          > "$R/gpurun_out/$out.log" 2>&1); rc=$?; echo "== $out rc=$rc"; tail -2 "gpurun_out/$out.log"; [[ $rc -le 1 ]] || exit $rc ;;
    *=*) run "${LIMIT:-300}" "${s%%=*}" bash -c "${s#*=}" ;;  # ad-hoc step: name=command
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
