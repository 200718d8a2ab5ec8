#!/bin/bash
# SQ instruction/wait counters + FETCH_SIZE for deep temporal-blocking variants (one rocprofv3 pass
# per counter group and variant, --kernel-trace only).
#   scripts/pmc_tbk.sh "<variant>;<variant>..."   -> gpurun_out/pmc_tbk/<tag>_p<i>/
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT="$R/gpurun_out/pmc_tbk"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra VS <<< "$1"
for v in "${VS[@]}"; do
  tag=$(echo "$v" | tr ',=' '__')
  i=0
  for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "FETCH_SIZE" "SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"; do
    i=$((i+1))
    echo "== $v pass $i: $grp"
    # shellcheck disable=SC2086
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/${tag}_p$i" -o run -- python3 "$R/bench/kernel_ab.py" --n 1024 --iters 3 --rounds 1 --variants "$v" > "$OUT/${tag}_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/${tag}_p$i.log"; exit 1; }
  done
done
