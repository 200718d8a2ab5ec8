#!/bin/bash
# Round 5, session D: effective clock and SQ ratios per heat7_wxk dispatch of the driver-form bench
# (eager, so every sweep is its own dispatch), one counter pass (--kernel-trace only).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05d
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES \
   SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU --kernel-trace \
   --output-format csv -d "$R/$O/clock" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --graph off \
   > "$R/$O/clock.log" 2>&1) || { tail -5 $O/clock.log; exit 1; }
python3 scripts/pmc_clock.py $O/clock/* > $O/clock.txt 2>&1 || find $O/clock | head
tail -30 $O/clock.txt
# x-geometry probe for the 27-point at 512-cell rows: box27_wxk with rows that fill whole x segments
# (fp32 496 = 2 x 248, fp64 480 = 4 x 120) against 512 (3 and 5 segments)
timeout -k 10 200 python bench/kernel_ab.py --kind box27 --n 512 --iters 10 --rounds 3 --variants "STEPS=3;STEPS=2;STEPS=3,EXP=16" \
  > $O/b27_f32_512.log 2>&1 && tail -3 $O/b27_f32_512.log &&
timeout -k 10 200 python bench/kernel_ab.py --kind box27 --n 512 --nx 496 --iters 10 --rounds 3 --variants "STEPS=3;STEPS=2" \
  > $O/b27_f32_496.log 2>&1 && tail -3 $O/b27_f32_496.log &&
timeout -k 10 200 python bench/kernel_ab.py --kind box27 --n 512 --dtype f64 --iters 10 --rounds 3 --variants "STEPS=3" \
  > $O/b27_f64_512.log 2>&1 && tail -2 $O/b27_f64_512.log &&
timeout -k 10 200 python bench/kernel_ab.py --kind box27 --n 512 --nx 480 --dtype f64 --iters 10 --rounds 3 --variants "STEPS=3" \
  > $O/b27_f64_480.log 2>&1 && tail -2 $O/b27_f64_480.log
