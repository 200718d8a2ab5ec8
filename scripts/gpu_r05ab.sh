#!/bin/bash
# Round 5, session AB: the K = 5 sweep with three window buffers (the DMA two planes ahead, one
# barrier per plane; MDFX_H7_NB3=1) against two: bitwise on odd shapes, kernel A/B, driver form.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ab
mkdir -p $O
for shp in "--nx 300 --ny 77 --nz 41" "--nx 1000 --ny 333 --nz 64" "--nx 1030 --ny 50 --nz 13"; do
  timeout -k 10 200 python bench/kernel_ab.py --kind heat7 $shp --iters 2 --rounds 1 \
    --variants "STEPS=5;STEPS=5,NB3=1" > $O/ab_odd.log 2>&1 || { tail -20 $O/ab_odd.log; exit 1; }
  tail -2 $O/ab_odd.log
done
for shp in "--n 1024" "--nx 1024 --ny 1024 --nz 128" "--n 512"; do
  tag=$(echo $shp | tr -d ' -')
  timeout -k 10 300 python bench/kernel_ab.py --kind heat7 $shp --iters 10 --rounds 4 \
    --variants "STEPS=5;STEPS=5,NB3=1" > $O/ab_$tag.log 2>&1 || { tail -20 $O/ab_$tag.log; exit 1; }
  echo "== $shp"; tail -2 $O/ab_$tag.log
done
for e in 0 1 0 1; do
  if [ $e = 1 ]; then export MDFX_H7_NB3=1; else unset MDFX_H7_NB3; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_$e.json 2> $O/drv_$e.err || { tail -5 $O/drv_$e.err; exit 1; }
  echo "drv nb3=$e $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], c['graph'], c['verified']['max_abs_diff'])" $O/drv_$e.json)"
done
