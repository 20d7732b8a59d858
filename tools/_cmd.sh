#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r01d
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_boussinesq.py > gpurun_out/r01d/bous.log 2>&1 || { tail -30 gpurun_out/r01d/bous.log; exit 1; }
tail -8 gpurun_out/r01d/bous.log
timeout -k 10 300 python bench.py > gpurun_out/r01d/bench.json 2> gpurun_out/r01d/bench.err && cat gpurun_out/r01d/bench.json
