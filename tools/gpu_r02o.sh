set -o pipefail
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 1150 python -u tools/bous_solve.py --ne 48 --P 8 --Ra 1e5 --x0 ckpt/bous_48_10000.npy --ckpt $O/ckpt --out $O/b48.json > $O/b48.log 2>&1; rc=$?
grep -v "  GMRES [0-9]" $O/b48.log | tail -8 | cut -c1-600
exit $rc
