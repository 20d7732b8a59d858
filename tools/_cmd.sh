#!/bin/bash
set -o pipefail
O=gpurun_out/r01o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_dist.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -5 $O/tests.log
