set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
rc=0
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/velocity_bench.py --ne 16 --P 8 --Re 1000 > $O/vb16.log 2>&1 || { tail -20 $O/vb16.log; exit 1; }
tail -1 $O/vb16.log
timeout -k 10 400 python -u tools/velocity_bench.py --ne 32 --P 8 --Re 1000 --reps 10 > $O/vb32.log 2>&1 || { tail -20 $O/vb32.log; exit 1; }
tail -1 $O/vb32.log
timeout -k 10 500 python -u tools/velocity_bench.py --ne 48 --P 8 --Re 1000 --reps 5 > $O/vb48.log 2>&1 || { tail -20 $O/vb48.log; exit 1; }
tail -1 $O/vb48.log
