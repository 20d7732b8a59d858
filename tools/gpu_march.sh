#!/bin/bash
# March-kernel iteration: parity/bitwise tests of the band variants, then in-process A/B.
set -o pipefail
O=gpurun_out/march
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_apply.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "march or variants or fused_apply" > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_env.py --var SEM_BAND_TILE --values 3,4,7,8 --meshes 8:64,8:256,8:512,8:1024,12:128 > $O/ab_tile.log 2>&1 || exit $?
grep -v amdgpu.ids $O/ab_tile.log
for WG in 512 1024 1536 2048 4096; do
  SEM_BAND_TILE=8 SEM_MARCH_WG=$WG timeout -k 10 120 python -u tools/ab_env.py --var SEM_BAND_CPOL --values 256 --meshes 8:1024 --rounds 3 > $O/wg$WG.log 2>&1 || exit $?
  echo "WG=$WG $(grep -v amdgpu.ids $O/wg$WG.log)"
done
