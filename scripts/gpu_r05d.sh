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
