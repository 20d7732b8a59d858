set -o pipefail
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 400 python -u tools/bous_solve.py --ne 16 --P 8 --Ra 1e4 --continuation 1e3 --iprint 2 --out $O/b16.json > $O/b16.log 2>&1; rc=$?
grep -v "  GMRES [0-9]" $O/b16.log | tail -40 | cut -c1-250
exit $rc
