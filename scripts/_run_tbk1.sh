set -o pipefail
cd $GRAFT_REPO_ROOT
S=scripts/gpu_step.sh
$S 400 gpurun_out/tbk_tests.log -- python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_temporal.py -k "heat7_deep or deep_temporal_3d"
rc=$?; [ $rc -ge 2 ] && exit $rc
$S 500 gpurun_out/ab_tbk.log -- python -u bench/kernel_ab.py --kind heat7 --n 1024 --iters 10 --rounds 3 --variants "STEPS=2;STEPS=2,TBK2=1,TBKRY=4;STEPS=2,TBK2=1,TBKRY=3;STEPS=2,TBK2=1,TBKRY=2;STEPS=3,TBKRY=2;STEPS=3,TBKRY=1;STEPS=3,TBKRY=3;STEPS=4,TBKRY=2" --json gpurun_out/ab_tbk.json
