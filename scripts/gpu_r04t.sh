#!/bin/bash
# Round 4, session T: halo-stream priority (MDFX_HALO_PRIORITY 1 = high, the round-4 default, vs 0 =
# normal) on the rank proxies, the 2-process shared-GPU ipc bench and the 4-process shared-GPU bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/t
v() { python -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" "$1"; }
for rep in 1 2; do
  for pr in 1 0; do
    for n in 8 4; do
      MDFX_HALO_PRIORITY=$pr timeout -k 10 200 python bench.py --rank-proxy $n --steps 48 --warmup 12 \
        > gpurun_out/t/p${n}_pr${pr}_$rep.json 2> gpurun_out/t/p${n}_pr${pr}_$rep.err || { tail -5 gpurun_out/t/p${n}_pr${pr}_$rep.err; exit 1; }
      echo "proxy$n prio$pr rep$rep $(v gpurun_out/t/p${n}_pr${pr}_$rep.json)"
    done
    MDFX_HALO_PRIORITY=$pr timeout -k 10 300 python bench.py --n 1024 --steps 48 --warmup 12 --gpus 2 --share-gpu --transport ipc \
      > gpurun_out/t/ipc2_pr${pr}_$rep.json 2> gpurun_out/t/ipc2_pr${pr}_$rep.err || { tail -5 gpurun_out/t/ipc2_pr${pr}_$rep.err; exit 1; }
    echo "ipc2 prio$pr rep$rep $(v gpurun_out/t/ipc2_pr${pr}_$rep.json)"
  done
done
