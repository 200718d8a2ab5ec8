#!/bin/bash
# Round 5, session P: single-slab steps without the exchange event wait: engine / CLI / proxy tests,
# a kernel trace of the eager driver form (gaps between sweeps), the driver form x3.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_cli.py \
  tests/test_gpu_proxy.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace1" -o run \
  -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --graph off > "$R/$O/trace1.log" 2>&1) || { tail -5 $O/trace1.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.json 2> $O/drv_$i.err || { tail -5 $O/drv_$i.err; exit 1; }
  echo "drv $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], c['graph'], [(t['graph'], t['ms_per_step']) for t in c['trials']], r['pct_of_measured_copy'], c['verified']['max_abs_diff'])" $O/drv_$i.json)"
done
