set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_abi.py tests/test_gpu_ns_velocity.py tests/test_gpu_solvers.py tests/test_gpu_boussinesq.py tests/test_gpu_dist.py "tests/test_gpu_apply.py::test_cfg5_checksums_full_size" tests/test_gpu_apply.py -k "position or cfg5 or ns or abi or solver or bous or dist or sweeps or tuning or launchers or cd or helmholtz" > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u tools/ns_solve.py --ne 16 --P 8 --Re 1000 --continuation 100,400 --out $O/ns16_1000.json > $O/ns16_1000.log 2>&1 || { tail -20 $O/ns16_1000.log; exit 1; }
tail -4 $O/ns16_1000.log
