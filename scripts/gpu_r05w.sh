#!/bin/bash
# Round 5, session W: K = 5 sweep with non-volatile row pins (rows interleave, hiding the packed-op
# dependency nops; MDFX_H7_NAR=1) against the shipped pins: bitwise and kernel A/B at 1024^3 / slabs.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 200 python bench/kernel_ab.py --kind heat7 --nx 300 --ny 77 --nz 41 --iters 2 --rounds 1 \
  --variants "STEPS=5;STEPS=5,NAR=1" > $O/ab_odd.log 2>&1 || { tail -20 $O/ab_odd.log; exit 1; }
tail -2 $O/ab_odd.log
for shp in "--n 1024" "--nx 1024 --ny 1024 --nz 128"; do
  tag=$(echo $shp | tr -d ' -')
  timeout -k 10 300 python bench/kernel_ab.py --kind heat7 $shp --iters 10 --rounds 4 \
    --variants "STEPS=4;STEPS=5;STEPS=5,NAR=1" > $O/ab_$tag.log 2>&1 || { tail -20 $O/ab_$tag.log; exit 1; }
  echo "== $shp"; tail -3 $O/ab_$tag.log
done
