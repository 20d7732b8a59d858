#!/bin/bash
# cfg5 end to end: the element-partitioned Boussinesq coupler at 128^2, P = 12 (9.45 M coupled DOFs), JNK
# from rest through Ra = 1e3 to Ra = 1e4, two ranks sharing the one GPU over gloo (rank 0 also holds the whole-mesh
# counterparts that solve the Newton updates).
set -o pipefail
O=gpurun_out/r02c6; mkdir -p $O
timeout -k 10 800 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29615 \
  tools/bous_cfg5_solve.py --backend gloo --Ra 1e4 --continuation 1e3 --out $O/cfg5_ra1e4.json > $O/cfg5.log 2>&1; rc=$?
grep -v "GMRES: [0-9]" $O/cfg5.log | tail -8 | cut -c1-700
exit $rc
