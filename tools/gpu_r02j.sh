set -o pipefail
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_krylov.py tests/test_gpu_solvers.py tests/test_gpu_boussinesq.py tests/test_gpu_ns_velocity.py tests/test_gpu_abi.py > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/sweep_bench.py > $O/sweep.log 2>&1 || { tail -5 $O/sweep.log; exit 1; }
tail -4 $O/sweep.log
timeout -k 10 300 python -u tools/bous_solve.py --ne 16 --P 8 --Ra 1e4 --continuation 1e3 --out $O/b16.json > $O/b16.log 2>&1 || { grep -v "  GMRES" $O/b16.log | tail -20; exit 1; }
grep '"Ra"' $O/b16.log | cut -c1-400
