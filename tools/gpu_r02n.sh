set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_apply.py tests/test_gpu_abi.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u tools/ab_env.py --var SEM_BAND_TILE --values 0,9,3 --meshes 8:64,8:256,8:1024,12:128 --rounds 7 > $O/ab_smem.log 2>&1 || { tail -5 $O/ab_smem.log; exit 1; }
cat $O/ab_smem.log
