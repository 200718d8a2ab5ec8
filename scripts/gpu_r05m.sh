#!/bin/bash
# Round 5, session M: SQ counters of the 27-point whole-row sweep at 512^3 fp32 (LDS issue, waits and
# bank conflicts next to VALU) and of the overlapping-segment sweep at 1024^3 for comparison.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05m
mkdir -p $O
pass() {  # pass <name> <kernel_ab args...>
  local name=$1
  shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES \
     SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_LDS --kernel-trace \
     --output-format csv -d "$R/$O/$name" -o run -- python3 "$R/bench/kernel_ab.py" --kind box27 --iters 10 --rounds 1 "$@" \
     > "$R/$O/$name.log" 2>&1) || { tail -5 $O/$name.log; exit 1; }
  echo "== $name"; grep -E "STEPS" $O/$name.log | tail -1
  python3 scripts/pmc_sq.py $O/$name box27_wxk > $O/$name.txt 2>&1; cat $O/$name.txt
}
pass wr512 --n 512 --variants "STEPS=3" &&
pass ov1024 --n 1024 --iters 4 --variants "STEPS=3"
