#!/bin/bash
set -o pipefail
O=gpurun_out/r01l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_apply.py -k "variants" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/ab_env.py --var SEM_BAND_TILE --values 4,3,5,6 --meshes 8:64,8:512,8:1024 --rounds 4 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
