#!/bin/bash
# Round evidence: bench JSON, rocprofv3 kernel trace/stats of the same bench command, and
# PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs) for the bench kernels.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
echo bench ok; cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python bench.py --cpu-seconds 0 > $OUT/trace.log 2>&1 || { echo trace failed; tail $OUT/trace.log; exit 1; }
echo trace ok
for PMC in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  N=$(echo $PMC | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $PMC -d $OUT/pmc_$N -o pmc --output-format csv -- python tools/kbench.py --meshes 8:64,8:1024 --reps 50 > $OUT/pmc_$N.log 2>&1 || { echo "pmc $N failed"; tail -3 $OUT/pmc_$N.log; }
done
echo done
