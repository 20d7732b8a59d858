#!/bin/bash
# round-6 GPU session: suite, bench, PMC passes of the band kernel (cfg2 and 1024^2).  Stops at the first failure.
set -o pipefail
O=gpurun_out/${1:-r06b}; mkdir -p $O
STEPS=${STEPS:-suite bench pmc}
for s in $STEPS; do
  case $s in
  suite) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/suite.log 2>&1 \
           || { echo "suite failed"; tail -30 $O/suite.log; exit 1; }; tail -3 $O/suite.log ;;
  rccl) timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -x -v -s --timeout 450 --timeout-method thread > $O/rccl.log 2>&1 \
           || { echo "rccl failed"; tail -30 $O/rccl.log; exit 1; }; tail -3 $O/rccl.log ;;
  bench) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
           || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }; cut -c1-600 $O/bench.json ;;
  pmc) bash tools/pmc_run.sh $O/pmc64 -- python tools/kbench.py --meshes 8:64 --reps 50 && \
       bash tools/pmc_run.sh $O/pmc1024 -- python tools/kbench.py --meshes 8:1024 --reps 5 || exit 1 ;;
  esac
done
