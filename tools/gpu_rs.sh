#!/bin/bash
# Row-staging iteration: bitwise/parity tests of the band variants, then in-process A/B.
set -o pipefail
O=gpurun_out/rs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_apply.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "march or variants or fused_apply" > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_env.py --var SEM_BAND_TILE --values 3,4,9,10 --meshes 8:64,8:256,8:1024,12:128 --rounds 7 > $O/ab_tile.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_tile.log
