set -o pipefail
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 170 python -u tools/recycle_probe.py 8 > $O/probe8.log 2>&1; rc=$?
cat $O/probe8.log | tail -18
exit $rc
