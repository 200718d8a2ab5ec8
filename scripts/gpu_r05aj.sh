#!/bin/bash
# Round 5, session AJ: bench.py after the pencil-depth refactor (depth_for_layout): the 4-process
# headline-size ipc test (slab and pencil gates), the proxy tests, the bench tests, the default form.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05aj
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipc.py -k "headline_size or bench" \
  tests/test_gpu_proxy.py tests/test_gpu_cli.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/default.json 2> $O/default.err || { tail -5 $O/default.err; exit 1; }
grep -o '"value": [0-9.]*\|"temporal_block": [0-9]*' $O/default.json
timeout -k 10 300 python bench.py --rank-proxy 8 --py 2 --steps 48 --warmup 12 > $O/pencil8.json 2> $O/pencil8.err || { tail -5 $O/pencil8.err; exit 1; }
grep -o '"value": [0-9.]*\|"temporal_block": [0-9]*' $O/pencil8.json
