#!/bin/bash
# cfg4 (Boussinesq JNK, 48^2, P=8) continuation in Ra on the device, stage 1: Ra = 1e3, 1e4, 1e5
# (each stage checkpointed; a stage cut by the time limit resumes from its last Newton state).
set -o pipefail
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 1140 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e5 --continuation 1e3,1e4 --iprint 2 --ckpt $O/ckpt --out $O/b48.json > $O/b48.log 2>&1; rc=$?
grep -v "  GMRES [0-9]\|block-Jacobi" $O/b48.log | tail -12 | cut -c1-400
exit $rc
