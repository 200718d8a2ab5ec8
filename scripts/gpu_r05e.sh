#!/bin/bash
# Round 5, session E: effective clock (GRBM_GUI_ACTIVE / 8 XCDs / dispatch time) and SQ ratios of the
# 27-point sweeps at 512^3 fp32: overlapping x segments (3 per row), whole-row blocks with LDS x edges
# (MDFX_WXK_EXP=16), and the 496-cell rows that fill 2 overlapping segments; one counter pass each.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05e
mkdir -p $O
pass() {  # pass <name> <kernel_ab args...>
  local name=$1
  shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES \
     SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU --kernel-trace \
     --output-format csv -d "$R/$O/$name" -o run -- python3 "$R/bench/kernel_ab.py" --kind box27 --iters 10 --rounds 1 "$@" \
     > "$R/$O/$name.log" 2>&1) || { tail -5 $O/$name.log; exit 1; }
  echo "== $name"; tail -2 $O/$name.log
  python3 scripts/pmc_clock.py $O/$name box27_wxk > $O/$name.txt 2>&1; tail -4 $O/$name.txt
}
pass ov512 --n 512 --variants "STEPS=3" &&
pass wr512 --n 512 --variants "STEPS=3,EXP=16" &&
pass ov496 --n 512 --nx 496 --variants "STEPS=3"
