#!/bin/bash
# cfg4 (Boussinesq JNK, 48^2, P=8) continuation stage 2: from the Ra = 1e5 solution (ckpt/) through
# Ra = 3e5 to Ra = 1e6; every Newton step checkpointed under gpurun_out/r02v/ckpt.
set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 1140 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --continuation 3e5 --x0 ckpt/bous_48_100000.npy --iprint 2 --ckpt $O/ckpt --out $O/b48.json > $O/b48.log 2>&1; rc=$?
grep -v "  GMRES [0-9]\|block-Jacobi" $O/b48.log | tail -12 | cut -c1-400
exit $rc
