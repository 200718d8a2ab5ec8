#!/bin/bash
# Hardware counters of the tuned kernels through the A/B harness, one rocprofv3 pass per counter
# group, --kernel-trace only (no sys/runtime trace with --pmc).
#   scripts/pmc_profile.sh [TAG] [kernel_ab.py args]     (default: heat7 1024^3 fp32, single + fused)
# Output: gpurun_out/pmc_<TAG>/p<i>/...; summarise with scripts/pmc_summary.py gpurun_out/pmc_<TAG> FIELD_BYTES
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-heat7}
shift || true
ARGS=${*:---n 1024 --iters 4 --rounds 1 --variants RY=2,PF=1;STEPS=2,TBRY=2}
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  echo "== $TAG pass $i: $grp"
  # shellcheck disable=SC2086
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/bench/kernel_ab.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
