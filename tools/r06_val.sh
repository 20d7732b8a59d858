O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/suite.log 2>&1 || { echo suite failed; tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -x -v -s --timeout 450 --timeout-method thread > $O/rccl.log 2>&1 || { echo rccl failed; tail -20 $O/rccl.log; exit 1; }
timeout -k 10 300 python tools/vsolve_probe.py --ab-edge 0 --ab-back 0 --out $O/vsolve_cfg5.json > $O/vsolve.log 2>&1 || { echo vsolve failed; tail -5 $O/vsolve.log; exit 1; }
tail -3 $O/vsolve.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
echo ok
