#!/bin/bash
# Run GPU steps in order; a step that crashes, aborts or times out (exit >= 124, or a signal) ends
# the script, a step that merely fails (exit 1, e.g. a failed assertion) lets the next one run.
#   scripts/gpu_step.sh <timeout_s> <log> -- cmd ...   (one step; exit code passed through)
t=$1; log=$2; shift 3
echo "[gpu_step] $(date +%T) $*" >&2
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc -> $log" >&2
tail -3 "$log" >&2
exit $rc
