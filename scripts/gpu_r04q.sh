#!/bin/bash
# Round 4, session Q: fp64 K = 4 pencils (loopback, ipc, proxy GPU tests) and the hardware counters
# of the fp64 K = 4 heat7_wxk sweep (FETCH / WRITE / L2 / LDS / SQ passes at 1024^3).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py tests/test_gpu_ipc.py tests/test_gpu_proxy.py -k "pencil" \
  > gpurun_out/q/tests.log 2>&1 || { tail -30 gpurun_out/q/tests.log; exit 1; }
tail -1 gpurun_out/q/tests.log
bash scripts/pmc_profile.sh f64k4 --n 1024 --dtype f64 --iters 4 --rounds 1 --variants "STEPS=4" || exit 1
cd "$R"
python scripts/pmc_summary.py gpurun_out/pmc_f64k4 8589934592 > gpurun_out/q/pmc_f64k4.txt && cat gpurun_out/q/pmc_f64k4.txt
