#!/bin/bash
# Round 5, session AA: SQ counters of the K = 5 sweep (2-cell rows) against the K = 4 sweep at
# 1024^3: VALU issue, waits, instruction mix per plane step.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05aa
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES \
   SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --kernel-trace \
   --output-format csv -d "$R/$O/p1" -o run -- python3 "$R/bench/kernel_ab.py" --kind heat7 --n 1024 --iters 6 --rounds 1 \
   --variants "STEPS=4;STEPS=5" > "$R/$O/p1.log" 2>&1) || { tail -5 $O/p1.log; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES \
   SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace \
   --output-format csv -d "$R/$O/p2" -o run -- python3 "$R/bench/kernel_ab.py" --kind heat7 --n 1024 --iters 6 --rounds 1 \
   --variants "STEPS=4;STEPS=5" > "$R/$O/p2.log" 2>&1) || { tail -5 $O/p2.log; exit 1; }
for p in p1 p2; do for k in "heat7_wxk<float, 3, 2, 4" "heat7_wxk<float, 5, 4, 5"; do
  echo "== $p $k"; python3 scripts/pmc_sq.py $O/$p "$k" 2>&1 | tail -14; done; done
