#!/bin/bash
# Hardware counters for the headline kernels (1024^3 fp32): single-sweep heat7_zw and fused heat7_tb2.
# One rocprofv3 pass per counter group, --kernel-trace only (no sys/runtime trace with --pmc).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
APP="$R/bench/kernel_ab.py --n 1024 --iters 4 --rounds 1 --variants RY=2,PF=1;STEPS=2,TBRY=2"
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters_list.txt" 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 $APP > "$R/gpurun_out/pmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc/p$i.log"; }
done
ls -R "$R/gpurun_out/pmc" | head -40
