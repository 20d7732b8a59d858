#!/bin/bash
# Strip-partitioned NS (ABI 5 strip sem_ns_apply) and the NS / velocity-solve suites on the device, then
# cfg4 (Boussinesq JNK, 48^2, P=8) final stage Ra = 1e6 from the Ra = 3e5 solution of r02y.
set -o pipefail
O=gpurun_out/r02z; mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_ns_apply.py tests/test_gpu_ns_velocity.py tests/test_gpu_solvers.py -k "ns or NS or partitioned or velocity or gemv" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --x0 ckpt/bous_48_300000.npy --iprint 2 --ckpt $O/ckpt --out $O/b48.json > $O/b48.log 2>&1; rc=$?
grep "^{\|^Newton\|checkpoint" $O/b48.log | tail -14 | cut -c1-400
exit $rc
