#!/bin/bash
# Quick kernel iteration: GPU parity tests + kernel micro-benchmark.
set -o pipefail
TAG=${1:-iter}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?; echo "gputests rc=$rc"; tail -6 gpurun_out/${TAG}_gputests.log
[ $rc -gt 1 ] && exit $rc
for ALGO in ${ALGOS:-1 2 3}; do
timeout -k 10 300 python tools/kbench.py --algo $ALGO ${KB_ARGS} > gpurun_out/${TAG}_kbench_a$ALGO.log 2>&1
rc=$?; echo "kbench algo=$ALGO rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_kbench_a$ALGO.log
[ $rc -ne 0 ] && exit $rc
done
exit $rc
