set -o pipefail
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 500 python -u tools/bous_solve.py --ne 16 --P 8 --Ra 1e4 --continuation 1e3 --out $O/b16.json > $O/b16.log 2>&1 || { grep -v "  GMRES" $O/b16.log | tail -20; exit 1; }
grep '"Ra"' $O/b16.log
