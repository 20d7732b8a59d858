#!/bin/bash
# ABI 6 (column-ranged sem_velocity_blocks, column-chunked velocity factorisation): host/ABI, velocity
# and solver suites on the device, then cfg5's NS update on one GPU (tools/cfg5_ns_probe.py).
set -o pipefail
O=gpurun_out/r02q2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_ns_velocity.py tests/test_gpu_solvers.py tests/test_gpu_abi.py tests/test_components.py tests/test_gpu_boussinesq.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 540 python -u tools/cfg5_ns_probe.py > $O/cfg5_ns.log 2>&1; rc=$?
tail -4 $O/cfg5_ns.log | cut -c1-700
exit $rc
