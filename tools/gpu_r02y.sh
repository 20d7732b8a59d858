#!/bin/bash
# Component counterparts + the fixed partitioned-solver test on the device, then cfg4 (Boussinesq JNK,
# 48^2, P=8) from rest through Ra = 1e3, 1e4, 1e5, 3e5 towards 1e6 with every Newton step
# checkpointed under gpurun_out/r02y/ckpt (the run is cut by its own time limit and resumed).
set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_components.py tests/test_gpu_dist.py tests/test_gpu_ns_apply.py tests/test_gpu_abi.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 960 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --continuation 1e3,1e4,1e5,3e5 --iprint 2 --ckpt $O/ckpt --out $O/b48.json > $O/b48.log 2>&1; rc=$?
grep -v "  GMRES [0-9]\|block-Jacobi" $O/b48.log | tail -12 | cut -c1-400
exit $rc
