#!/bin/bash
# Kernarg-preload iteration: GPU parity suite, then in-process A/B of SEM_BAND_KP.
set -o pipefail
O=gpurun_out/kp
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_env.py --var SEM_BAND_KP --values 0,1 --meshes 8:64,8:256,8:1024,12:128 --rounds 9 > $O/ab.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab.log
