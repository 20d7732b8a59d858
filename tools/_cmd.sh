#!/bin/bash
set -o pipefail
O=gpurun_out/r01g
mkdir -p $O
timeout -k 10 300 python -u tools/ab_env.py --var SEM_BAND_TILE --values 0,1,2 --meshes 8:64,8:256,8:1024 --rounds 5 > $O/tile.log 2>&1 || { tail -20 $O/tile.log; exit 1; }
cat $O/tile.log
for D in 0 16 48 112; do
  SEM_DIAG=$D timeout -k 10 120 python -u tools/kbench.py --meshes 8:64 --reps 400 > $O/diag$D.log 2>&1 || { tail -5 $O/diag$D.log; exit 1; }
  echo "SEM_DIAG=$D: $(grep 'P= 8' $O/diag$D.log)"
done
