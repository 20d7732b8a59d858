#!/bin/bash
# Fused nested-interior solve (ns_condense.hip): parity, velocity-solve / Schur-matvec timings at
# 32^2 and 48^2, kernel trace at 48^2.
set -o pipefail
O=gpurun_out/r02w; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_ns_velocity.py tests/test_gpu_solvers.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/velocity_bench.py --ne 32 --P 8 --configs nested:cr > $O/vb32.log 2>&1 || { tail -5 $O/vb32.log; exit 1; }
tail -1 $O/vb32.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python -u tools/velocity_bench.py --ne 48 --P 8 --configs nested:cr > $O/vb48.log 2>&1 || { tail -5 $O/vb48.log; exit 1; }
grep "{" $O/vb48.log | tail -1 | cut -c1-600
