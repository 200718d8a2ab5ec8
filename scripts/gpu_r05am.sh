#!/bin/bash
# Round 5, session AM: the rank proxies with the SDMA pulls (--transport ipc_sdma -> proxy_sdma: no
# CUs taken from the interior sweep) against the blit pulls, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05am
mkdir -p $O
for i in 1 2; do for t in auto ipc_sdma; do for n in 8 4; do
  timeout -k 10 300 python bench.py --rank-proxy $n --transport $t --steps 50 --warmup 10 > $O/p${n}_${t}_$i.json 2> $O/p${n}_${t}_$i.err || { tail -5 $O/p${n}_${t}_$i.err; exit 1; }
  echo "p$n $t $(grep -o '"value": [0-9.]*' $O/p${n}_${t}_$i.json)"
done; done; done
