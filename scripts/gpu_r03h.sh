#!/bin/bash
# Round 3 session H: heat7_wxk K = 4 (2-row waves) as the fp32 default -- GPU tier of the temporal
# and engine tests, smoke, then the configs and counters.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --steps 48 --warmup 12"
scripts/gpu_session.sh "temporal=$PYT tests/test_gpu_temporal.py tests/test_gpu_engine.py tests/test_gpu_proxy.py" smoke || exit $?
grep -q ' passed' gpurun_out/temporal.log && ! grep -q 'failed' gpurun_out/temporal.log || { tail -30 gpurun_out/temporal.log; exit 1; }
scripts/gpu_session.sh "d1=$B" "drv1=python bench.py --steps 20 --warmup 5" "k3=$B --temporal 3" "wb4=MDFX_WTK_WB=4 $B" \
  "d2=$B" "drv2=python bench.py --steps 20 --warmup 5" "dflt=python bench.py" \
  "n512=$B --n 512" "n512k3=$B --n 512 --temporal 3" \
  "p2=python bench.py --rank-proxy 2 --steps 48 --warmup 12" "p4=python bench.py --rank-proxy 4 --steps 48 --warmup 12" \
  "p8=python bench.py --rank-proxy 8 --steps 48 --warmup 12" "p8k3=python bench.py --rank-proxy 8 --steps 48 --warmup 12 --temporal 3" \
  "v8=$B --virtual-ranks 8" "n3072=python bench.py --n 3072 --steps 12 --warmup 4" \
  "f64=$B --dtype f64" "f64wxk=MDFX_H7_WXK=1 $B --dtype f64" \
  "f64r=python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12" \
  "f64rwxk=MDFX_H7_WXK=1 python bench.py --n 2048 --dtype f64 --steps 24 --warmup 3 --residual-every 12" || exit $?
scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
for f in d1 drv1 k3 wb4 d2 drv2 dflt n512 n512k3 p2 p4 p8 p8k3 v8 n3072 f64 f64wxk f64r f64rwxk; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log)"; done
