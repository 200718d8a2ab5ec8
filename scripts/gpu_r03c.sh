#!/bin/bash
# Round 3 session C: natural-layout jacobi5_tbk (modes 0/1/2, fp32 and reference precision),
# heat7_wtk recheck, rank-proxy tests and runs at N = 2/4/8, counter passes.
set -o pipefail
cd "$(dirname "$0")/.."
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
B="python bench.py --steps 48 --warmup 16"
M="$B --stencil jacobi5 --n 16384"
steps=("temporal=$PYT tests/test_gpu_temporal.py" "proxytests=$PYT tests/test_gpu_proxy.py")
for r in a b; do
  for m in 0 1 2; do steps+=("mdf_nat${m}_$r=MDFX_J5_NAT=$m $M"); done
  for m in 0 1 2; do steps+=("mdfref_nat${m}_$r=MDFX_J5_NAT=$m $M --ref-precision"); done
done
for r in a b; do
  for m in 0 1; do steps+=("b27f32_nat${m}_$r=MDFX_B27_NAT=$m $B --stencil box27 --n 512"); done
done
steps+=("mdf_f64=$M --dtype f64" "mdf_dialogue=printf '100\n16384\n16384\n' | ./build/bin/mdf --json")
steps+=("h1024_a=$B" "h1024_drv=python bench.py --steps 20 --warmup 5")
for n in 2 4 8; do steps+=("proxy$n=python bench.py --rank-proxy $n --steps 48 --warmup 12"); done
steps+=("proxy8_nosplit=MDFX_WTK_SPLIT=-1 python bench.py --rank-proxy 8 --steps 48 --warmup 12"
        "proxy4_nosplit=MDFX_WTK_SPLIT=-1 python bench.py --rank-proxy 4 --steps 48 --warmup 12"
        "proxy8_nofuse=MDFX_FUSE_REGIONS=0 python bench.py --rank-proxy 8 --steps 48 --warmup 12"
        "v8=$B --virtual-ranks 8" "v8_nosplit=MDFX_WTK_SPLIT=-1 $B --virtual-ranks 8")
steps+=("proxy8_r0=python bench.py --rank-proxy 8 --proxy-rank 0 --steps 48 --warmup 12"
        "slab128=python bench.py --nz 128 --steps 48 --warmup 12" "h1024_b=$B"
        "h512_k2=$B --n 512" "h512_k3=$B --n 512 --temporal 3")
LIMIT=400 scripts/gpu_session.sh "${steps[@]}" || exit $?
PMC_TAG=h1024 scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
PMC_TAG=proxy8 BENCH_ARGS="--rank-proxy 8" scripts/gpu_session.sh pmc_fetch pmc_write || exit $?
TAG=h1024 bash scripts/pmc_sq.sh || exit $?
for f in gpurun_out/mdf*.log gpurun_out/h1024*.log gpurun_out/proxy*.log gpurun_out/slab128.log; do
  echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"implied_node_gcells": [0-9.]*' $f)"; done
