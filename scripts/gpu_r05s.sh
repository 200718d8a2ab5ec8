#!/bin/bash
# Round 5, session S: the window rows by buffer LDS-DMA with a per-row descriptor (lanes and rows
# planes outside the storage read zeros without a fetch; A/B switch MDFX_BL_AB): bitwise
# tests with the switch on, kernel A/B, effective clock of both, the driver form interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05s
mkdir -p $O
MDFX_BL_AB=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_temporal.py \
  -k "heat7_wxk" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 4 \
  --variants "STEPS=4;STEPS=4,BL=1" > $O/ab_1024.log 2>&1 || { tail -20 $O/ab_1024.log; exit 1; }
tail -3 $O/ab_1024.log
for e in 0 1; do
  (cd /tmp && export TMPDIR=/tmp && if [ $e = 1 ]; then export MDFX_BL_AB=1; fi && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
     --kernel-trace --output-format csv -d "$R/$O/clk$e" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --graph off \
     > "$R/$O/clk$e.log" 2>&1) || { tail -5 $O/clk$e.log; exit 1; }
  echo "clock bl=$e"; python3 scripts/pmc_clock.py $O/clk$e "heat7_wxk<float, 3, 2, 4, 8" | tail -8
done
for e in 0 1 0 1 0 1 0 1; do
  if [ $e = 1 ]; then export MDFX_BL_AB=1; else unset MDFX_BL_AB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_$e.json 2> $O/drv_$e.err || { tail -5 $O/drv_$e.err; exit 1; }
  echo "drv bl=$e $(python -c "import json,sys; r=json.load(open(sys.argv[1])); c=r['config']; print(r['value'], c['graph'], c['verified']['max_abs_diff'])" $O/drv_$e.json)"
done
