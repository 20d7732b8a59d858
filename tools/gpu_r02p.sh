#!/bin/bash
# (1) 2-rank rehearsal of the driver's multi-GPU bench path on one GPU (gloo), both exchanges;
# (2) cfg4's Ra = 1e6 stage from the Ra = 3e5 state with the PCD Schur preconditioner (opt-in) -- the
#     mass-diagonal run of the same stage took 1,426 s over 5 Newton steps (r02z + r02z2).
set -o pipefail
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 \
  bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --hbm-ne 0 --cpu-seconds 0 > $O/bench2_gloo.json 2> $O/bench2_gloo.err || { tail -5 $O/bench2_gloo.err; exit 1; }
cut -c1-300 $O/bench2_gloo.json
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 \
  bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --hbm-ne 0 --cpu-seconds 0 --exchange p2p --scaling strong > $O/bench2_gloo_p2p.json 2> $O/bench2_gloo_p2p.err || { tail -5 $O/bench2_gloo_p2p.err; exit 1; }
cut -c1-300 $O/bench2_gloo_p2p.json
timeout -k 10 900 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --x0 ckpt/bous_48_300000.npy --schur-precond pcd --iprint 2 --ckpt $O/ckpt --out $O/b48_pcd.json > $O/b48_pcd.log 2>&1; rc=$?
grep "^{\|^Newton\|checkpoint" $O/b48_pcd.log | tail -12 | cut -c1-400
exit $rc
