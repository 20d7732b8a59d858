#!/bin/bash
# One GPU session: parity suite -> smoke -> the driver's bench command -> rocprofv3 kernel
# trace/stats of that same command.  Each GPU step has its own time limit; a failure, crash or
# timeout ends the session (no retries).  Output under gpurun_out/<tag>/.
set -o pipefail
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 5"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread \
  > $O/gputests.log 2>&1; rc=$?
tail -4 $O/gputests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python $BENCH > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python $BENCH \
  > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python tools/prof_summary.py $O > $O/prof_summary.txt 2>&1
head -30 $O/prof_summary.txt
exit $rc
