set -o pipefail
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 300 python -u tools/bous_solve.py --ne 8 --P 8 --Ra 1e6 --continuation 1e3,1e4,1e5 --out $O/b8.json > $O/b8.log 2>&1 || { tail -20 $O/b8.log; exit 1; }
grep '"Ra"' $O/b8.log; tail -1 $O/b8.log | cut -c1-300
timeout -k 10 600 python -u tools/bous_solve.py --ne 16 --P 8 --Ra 1e6 --continuation 1e3,1e4,1e5 --out $O/b16.json > $O/b16.log 2>&1 || { tail -20 $O/b16.log; exit 1; }
grep '"Ra"' $O/b16.log; tail -1 $O/b16.log | cut -c1-300
