#!/bin/bash
# Round 4 session H: host enqueue vs completion of the N = 8 proxy (bench/host_probe.py).
set -o pipefail
cd "$(dirname "$0")/.."
scripts/gpu_session.sh "hp8=python bench/host_probe.py" "hp8pen=python bench/host_probe.py --py 2" "hp4=python bench/host_probe.py --ranks 4" \
  "hp1=python bench/host_probe.py --ranks 1" || exit $?
cat gpurun_out/hp8.log gpurun_out/hp8pen.log gpurun_out/hp4.log gpurun_out/hp1.log | grep "^{"
nproc; cat /proc/cpuinfo | grep "model name" | head -1
