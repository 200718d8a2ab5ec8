#!/bin/bash
# Round 5, session AD: kernel timeline of the N = 8 rank proxy at K = 5 (eager, 1 round, overlapped):
# where the ~70 us per sweep beyond the interior sweep go.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05ad
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/p8" -o run -- \
  python3 "$R/bench.py" --rank-proxy 8 --steps 50 --warmup 10 --graph off --rounds 1 --overlap > "$R/$O/p8.log" 2>&1) \
  || { tail -5 $O/p8.log; exit 1; }
grep -o '"value": [0-9.]*' $O/p8.log
python3 scripts/timeline.py $O/p8/run_kernel_trace.csv > $O/timeline.txt && tail -40 $O/timeline.txt
