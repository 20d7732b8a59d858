#!/bin/bash
# Condensed direct-solve preconditioner for the CD Jacobian (ncomp=1 line condensation):
# GPU parity of the new pieces, CD solves at 32^2 / 64^2 against the plain device GMRES, and a
# Boussinesq 16^2 JNK probe.
set -o pipefail
O=gpurun_out/r02r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_ns_velocity.py tests/test_gpu_solvers.py tests/test_gpu_abi.py > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
grep -h "device CD solve\|cfg2 CD solve" $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/solve_bench.py --ne 32 --P 8 --oracle 0 --scipy 0 > $O/cd32.json 2>&1 || { tail -5 $O/cd32.json; exit 1; }
cat $O/cd32.json
timeout -k 10 300 python -u tools/solve_bench.py --ne 64 --P 8 --oracle 0 --scipy 0 > $O/cd64.json 2>&1 || { tail -5 $O/cd64.json; exit 1; }
cat $O/cd64.json
timeout -k 10 400 python -u tools/bous_solve.py --ne 16 --P 8 --Ra 1e4 --continuation 1e3 --out $O/b16.json > $O/b16.log 2>&1 || { tail -5 $O/b16.log; exit 1; }
grep -v "  GMRES [0-9]" $O/b16.log | tail -4 | cut -c1-700
