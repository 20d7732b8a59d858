set -o pipefail
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ns_apply.py tests/test_gpu_ns_velocity.py tests/test_host_api.py > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/velocity_bench.py --ne 32 --P 8 --Re 1000 --configs nested:cr,nested:thomas > $O/vb32.log 2>&1 || { tail -5 $O/vb32.log; exit 1; }
timeout -k 10 300 python -u tools/velocity_bench.py --ne 48 --P 8 --Re 1000 --configs nested:cr,nested:thomas > $O/vb48.log 2>&1 || { tail -5 $O/vb48.log; exit 1; }
tail -1 $O/vb48.log
tail -1 $O/vb32.log
timeout -k 10 400 python -u tools/ns_solve.py --ne 32 --P 8 --Re 1000 --continuation 100,400 --out $O/ns32_1000.json > $O/ns32.log 2>&1 || { tail -5 $O/ns32.log; exit 1; }
tail -4 $O/ns32.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_solvers.py > $O/tests_solvers.log 2>&1; rc=$?
tail -5 $O/tests_solvers.log
exit $rc
