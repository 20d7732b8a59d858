#!/bin/bash
# cfg4 (Boussinesq JNK, 48^2, P=8) Ra = 1e6 stage resumed from its Newton-2 state (r02z), every Newton
# step checkpointed; cut by its own time limit and resumed again if needed.
set -o pipefail
O=gpurun_out/r02z2; mkdir -p $O
timeout -k 10 1140 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --x0 ckpt/bous_48_1e6_newton2.npy --resume 1 --iprint 2 --ckpt $O/ckpt --out $O/b48.json > $O/b48.log 2>&1; rc=$?
grep "^{\|^Newton\|checkpoint" $O/b48.log | tail -14 | cut -c1-400
exit $rc
