set -o pipefail
cd $GRAFT_REPO_ROOT
S=scripts/gpu_step.sh
$S 300 gpurun_out/tbk_tests.log -- python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_engine.py tests/test_gpu_kernels.py || exit $?
$S 300 gpurun_out/bench_n1.json -- python bench.py --repeats 3 || exit $?
$S 300 gpurun_out/ab_1024.log -- python -u bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 3 --variants "STEPS=2;STEPS=3;STEPS=2,TBK2=0"
