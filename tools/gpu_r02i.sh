set -o pipefail
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 1100 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e4 --continuation 1e3 --ckpt $O/ckpt --out $O/b48.json > $O/b48.log 2>&1 || { grep -v "  GMRES" $O/b48.log | tail -20; exit 1; }
grep '"Ra"' $O/b48.log
