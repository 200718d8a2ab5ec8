#!/bin/bash
# Round 5, session AK: split ghost waits (the upper boundary after the hi ghosts, the interior after the lo ghosts)
# (ahead of the pulled signals and the waits for the neighbours' pulls): the ipc, proxy and
# multi-process tests, then the N = 2 / 4 / 8 proxies and the N = 8 proxy's timeline.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05ak
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipc.py \
  tests/test_gpu_proxy.py tests/test_gpu_multiprocess.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  echo "$tag $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], r['ms_per_step'], c.get('temporal_block'), r.get('measured_copy_TBps'))" $O/$tag.json)"; }
run p2 --rank-proxy 2 --steps 50 --warmup 10
run p4 --rank-proxy 4 --steps 50 --warmup 10
run p8 --rank-proxy 8 --steps 50 --warmup 10
run p8b --rank-proxy 8 --steps 50 --warmup 10
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/p8t" -o run -- \
  python3 "$R/bench.py" --rank-proxy 8 --steps 50 --warmup 10 --graph off --rounds 1 --overlap > "$R/$O/p8t.log" 2>&1) \
  || { tail -5 $O/p8t.log; exit 1; }
grep -o '"value": [0-9.]*' $O/p8t.log
python3 scripts/timeline.py $O/p8t/run_kernel_trace.csv 24 > $O/timeline.txt && cat $O/timeline.txt
