set -o pipefail
cd $GRAFT_REPO_ROOT
S=scripts/gpu_step.sh
$S 300 gpurun_out/xt_tests.log -- python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -m gpu -k xtiled || exit $?
$S 300 gpurun_out/ab_xt_f32.log -- python -u bench/kernel_ab.py --kind heat7 --nx 2048 --ny 512 --nz 256 --iters 20 --rounds 3 --variants "STEPS=1;STEPS=2;STEPS=2,XT=1;STEPS=2,XT=1,XRY=2;STEPS=2,XT=1,XRY=4" || exit $?
$S 300 gpurun_out/ab_xt_f64.log -- python -u bench/kernel_ab.py --kind heat7 --nx 1024 --ny 512 --nz 512 --dtype f64 --iters 10 --rounds 3 --variants "STEPS=1;STEPS=2;STEPS=2,XT=1;STEPS=2,XT=1,XRY=2;STEPS=2,XT=1,XRY=4"
