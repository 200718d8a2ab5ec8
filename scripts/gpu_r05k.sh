#!/bin/bash
# Round 5, session K: the single-step kernels after dropping their 1-row copies; the N = 8 / 4 rank
# proxies with graph replay on one / two / four hardware queues (DEBUG_HIP_FORCE_GRAPH_QUEUES) next to
# eager; a kernel trace of the eager N = 8 proxy for its timeline.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_temporal.py -k "not wxk and not wtk" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 8 4; do
  for q in 1 2 4; do
    DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 300 python bench.py --rank-proxy $n --steps 48 --warmup 12 \
      > $O/proxy${n}_q$q.json 2> $O/proxy${n}_q$q.err || { tail -5 $O/proxy${n}_q$q.err; exit 1; }
    echo "proxy $n q$q $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], c['graph'], [(t['graph'], t['min_rounds'], t['overlap'], t['ms_per_step']) for t in c['trials']])" $O/proxy${n}_q$q.json)"
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace8" -o run \
  -- python3 "$R/bench.py" --rank-proxy 8 --graph off --steps 24 --warmup 8 > "$R/$O/trace8.log" 2>&1) || { tail -5 $O/trace8.log; exit 1; }
tail -1 $O/trace8.log | cut -c1-200
