set -o pipefail
cd $GRAFT_REPO_ROOT
S=scripts/gpu_step.sh
export MDFX_DEBUG_ZC=1
$S 300 gpurun_out/tbk_tests.log -- python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_engine.py || exit $?
unset MDFX_DEBUG_ZC
$S 300 gpurun_out/bench_n1.json -- python bench.py --repeats 3 || exit $?
$S 300 gpurun_out/bench_v8.json -- python bench.py --virtual-ranks 8 --repeats 2 || exit $?
for nz in 128 256 512; do
$S 200 gpurun_out/ab_slab$nz.log -- python -u bench/kernel_ab.py --kind heat7 --nx 1024 --ny 1024 --nz $nz --iters 20 --rounds 3 --variants "STEPS=2;STEPS=2,TBK2=0;STEPS=3" --json gpurun_out/ab_slab_nz$nz.json || exit $?
done
