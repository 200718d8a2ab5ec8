set -o pipefail
cd $GRAFT_REPO_ROOT
S=scripts/gpu_step.sh
$S 600 gpurun_out/tbk_tests.log -- python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_engine.py tests/test_gpu_multiprocess.py tests/test_native.py -m gpu || exit $?
$S 300 gpurun_out/bench_n1.json -- python bench.py --repeats 2 || exit $?
$S 300 gpurun_out/bench_v8.json -- python bench.py --virtual-ranks 8 --repeats 2 || exit $?
$S 300 gpurun_out/ab_box27.log -- python -u bench/kernel_ab.py --kind box27 --n 512 --iters 20 --rounds 3 --variants "STEPS=2;STEPS=2,ZC=86;STEPS=2,ZC=128;STEPS=2,ZC=256;STEPS=2,ZC=32" || exit $?
$S 300 gpurun_out/ab_box27_f64.log -- python -u bench/kernel_ab.py --kind box27 --n 512 --dtype f64 --iters 10 --rounds 3 --variants "STEPS=2;STEPS=2,ZC=86;STEPS=2,ZC=128"
