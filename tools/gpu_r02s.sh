#!/bin/bash
# PCD Schur preconditioner: NS GPU parity (both preconditioners), cfg3 with each, Boussinesq 16^2.
set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -s -m gpu tests/test_gpu_ns_velocity.py tests/test_gpu_solvers.py tests/test_gpu_boussinesq.py > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
grep "schur_precond=" $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ns_solve.py --ne 32 --P 8 --Re 1000 --continuation 100,400 --schur-precond pcd --out $O/ns32_pcd.json > $O/ns32_pcd.log 2>&1 || { tail -5 $O/ns32_pcd.log; exit 1; }
grep "stage\|Ghia\|total" $O/ns32_pcd.log | tail -6
timeout -k 10 400 python -u tools/ns_solve.py --ne 32 --P 8 --Re 1000 --continuation 100,400 --schur-precond mass --out $O/ns32_mass.json > $O/ns32_mass.log 2>&1 || { tail -5 $O/ns32_mass.log; exit 1; }
grep "stage\|Ghia\|total" $O/ns32_mass.log | tail -6
timeout -k 10 400 python -u tools/bous_solve.py --ne 16 --P 8 --Ra 1e4 --continuation 1e3 --out $O/b16.json > $O/b16.log 2>&1 || { tail -5 $O/b16.log; exit 1; }
grep -v "  GMRES [0-9]" $O/b16.log | tail -2 | cut -c1-600
