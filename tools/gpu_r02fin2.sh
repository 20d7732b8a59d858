#!/bin/bash
# Round-2 final verification of the committed tree: full GPU suite -> smoke -> the driver's bench
# command -> rocprofv3 kernel trace of that command -> cfg5 partitioned coupled maps (1 rank over
# RCCL, 4 ranks on one GPU over gloo).  Each step has its own time limit; a failure ends the session.
set -o pipefail
O=gpurun_out/r02fin2
mkdir -p $O
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 5"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread \
  > $O/gputests.log 2>&1; rc=$?
tail -4 $O/gputests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python $BENCH > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python $BENCH \
  > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python tools/prof_summary.py $O > $O/prof_summary.txt 2>&1
head -8 $O/prof_summary.txt
timeout -k 10 300 python -u tools/bous_cfg5.py > $O/cfg5_1rank.json 2> $O/cfg5_1rank.err || { tail $O/cfg5_1rank.err; exit 1; }
cat $O/cfg5_1rank.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29621 \
  tools/bous_cfg5.py --backend gloo > $O/cfg5_4rank_gloo.json 2> $O/cfg5_4rank_gloo.err || { tail $O/cfg5_4rank_gloo.err; exit 1; }
cat $O/cfg5_4rank_gloo.json
