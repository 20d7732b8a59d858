set -o pipefail
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ns_velocity.py tests/test_gpu_solvers.py tests/test_gpu_boussinesq.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
for ne in 16 32 48; do
timeout -k 10 300 python -u tools/velocity_bench.py --ne $ne --P 8 --Re 1000 --reps 10 > $O/vb$ne.log 2>&1 || { tail -20 $O/vb$ne.log; exit 1; }
tail -1 $O/vb$ne.log
done
timeout -k 10 600 python -u tools/ns_solve.py --ne 32 --P 8 --Re 1000 --continuation 100,400 --out $O/ns32_1000.json > $O/ns32_1000.log 2>&1 || { tail -20 $O/ns32_1000.log; exit 1; }
tail -2 $O/ns32_1000.log | cut -c1-400
