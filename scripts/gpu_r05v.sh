#!/bin/bash
# Round 5, session V: the fp32 K = 5 sweep as the default: its bitwise tests (kernel, regions, engine,
# folded ipc), then the driver form and the N = 2 / 4 / 8 rank proxies at K = 5 against --temporal 4,
# and a kernel trace of the driver form.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_temporal.py \
  -k "wxk" > $O/t_temporal.log 2>&1 || { tail -30 $O/t_temporal.log; exit 1; }
tail -1 $O/t_temporal.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ipc.py \
  -k "k5 or k4_folded" tests/test_gpu_engine.py > $O/t_ipc_engine.log 2>&1 || { tail -30 $O/t_ipc_engine.log; exit 1; }
tail -1 $O/t_ipc_engine.log
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  echo "$tag $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], c.get('temporal'), c.get('parallelism'), r.get('measured_copy_TBps'), r.get('pct_of_measured_copy'), c.get('verified', {}).get('max_abs_diff') if isinstance(c.get('verified'), dict) else c.get('verified'))" $O/$tag.json)"; }
run drv5a --gpus 1 --steps 20 --warmup 5
run drv4a --gpus 1 --steps 20 --warmup 5 --temporal 4
run drv5b --gpus 1 --steps 20 --warmup 5
run drv4b --gpus 1 --steps 20 --warmup 5 --temporal 4
run p2 --rank-proxy 2 --steps 50 --warmup 10
run p4 --rank-proxy 4 --steps 50 --warmup 10
run p8 --rank-proxy 8 --steps 50 --warmup 10
run p8k4 --rank-proxy 8 --steps 48 --warmup 12 --temporal 4
run p4k4 --rank-proxy 4 --steps 48 --warmup 12 --temporal 4
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 > "$R/$O/prof.log" 2>&1) || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} head -6 {}
