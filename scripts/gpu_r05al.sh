#!/bin/bash
# Round 5, session AL: split ghost waits A/B at the N = 8 / 4 proxies, interleaved in one call
# (MDFX_NOSPLIT_AB=1: both ghost events before the boundary launch, as in session AF).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05al
mkdir -p $O
for i in 1 2 3; do for e in 0 1; do
  if [ $e = 1 ]; then export MDFX_NOSPLIT_AB=1; else unset MDFX_NOSPLIT_AB; fi
  timeout -k 10 300 python bench.py --rank-proxy 8 --steps 50 --warmup 10 > $O/p8_${e}_$i.json 2> $O/p8_${e}_$i.err || { tail -5 $O/p8_${e}_$i.err; exit 1; }
  echo "p8 nosplit=$e $(grep -o '"value": [0-9.]*' $O/p8_${e}_$i.json)"
done; done
for e in 0 1; do
  if [ $e = 1 ]; then export MDFX_NOSPLIT_AB=1; else unset MDFX_NOSPLIT_AB; fi
  timeout -k 10 300 python bench.py --rank-proxy 4 --steps 50 --warmup 10 > $O/p4_$e.json 2> $O/p4_$e.err || { tail -5 $O/p4_$e.err; exit 1; }
  echo "p4 nosplit=$e $(grep -o '"value": [0-9.]*' $O/p4_$e.json)"
done
