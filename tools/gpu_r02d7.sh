#!/bin/bash
# Checked, sliced batched inverse: velocity GPU tests, one-shot vs chunked CD condensation at P = 12,
# cfg5's whole-mesh CD update.
set -o pipefail
O=gpurun_out/r02d7; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ns_velocity.py -rf > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/chunk_probe.py --ne 32 --P 12 --chunks 0,6 > $O/p32.log 2>&1 || { tail -3 $O/p32.log; exit 1; }
grep "^{" $O/p32.log
timeout -k 10 300 python -u tools/chunk_probe.py --ne 64 --P 12 --chunks 0,6 > $O/p64.log 2>&1 || { tail -3 $O/p64.log; exit 1; }
grep "^{" $O/p64.log
timeout -k 10 300 python -u tools/cfg5_cd_probe.py > $O/cd.log 2>&1; rc=$?
grep "^{" $O/cd.log | cut -c1-400; tail -2 $O/cd.log | cut -c1-200
exit $rc
