#!/bin/bash
# Diagnose cfg5's CD update stagnation (r02c5): P = 12 condensation / nested-kernel / block-GEMV GPU tests,
# then the whole-mesh CD update at cfg5 (tools/cfg5_cd_probe.py).
set -o pipefail
O=gpurun_out/r02d5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ns_velocity.py -rf > $O/tests.log 2>&1; rc=$?
tail -8 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 420 python -u tools/cfg5_cd_probe.py > $O/cd.log 2>&1; rc=$?
grep "^{" $O/cd.log | cut -c1-400; tail -3 $O/cd.log | cut -c1-300
exit $rc
