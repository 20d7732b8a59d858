#!/bin/bash
# Round-2 re-verification of the committed tree on MI355X: GPU parity suite, smoke, the driver's
# bench command, and the rocprofv3 kernel trace/stats of that same command.
set -o pipefail
O=gpurun_out/r02q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 280 --timeout-method thread > $O/gputests.log 2>&1; rc=$?
tail -4 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
echo trace ok
