#!/bin/bash
# Round 4, session X: kernel traces of the N = 8 rank proxy with the SDMA exchange (proxy_sdma:
# face pulls on the copy engines, so no blit kernel of the runtime in the exchange) and with the
# default blit pulls, for the per-sweep timeline (scripts/kernel_timeline.py).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out/x"
cd /tmp && export TMPDIR=/tmp
for t in ipc_sdma ipc; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/x/$t" -o run -- \
    python3 "$R/bench.py" --rank-proxy 8 --transport $t --steps 24 --warmup 8 > "$R/gpurun_out/x/$t.log" 2>&1 \
    || { tail -20 "$R/gpurun_out/x/$t.log"; exit 1; }
  grep -o '"value": [0-9.]*' "$R/gpurun_out/x/$t.log" | head -1
done
