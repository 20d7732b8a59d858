#!/bin/bash
# One GPU session: parity tests -> smoke -> bench.  Each GPU step has its own time
# limit; a crash / abort / timeout (exit >= 124) ends the session (no retries).
set -o pipefail
TAG=${1:-r01}
STEPS=${STEPS:-2000}
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/${TAG}_${name}.log"
  return $rc
}
run gputests 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread
rc=$?; [ $rc -gt 1 ] && exit $rc
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 600 python bench.py --steps "$STEPS" --warmup 200 || exit $?
