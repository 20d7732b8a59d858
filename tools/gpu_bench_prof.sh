#!/bin/bash
# Round evidence: bench JSON, rocprofv3 kernel trace/stats of the same bench command, and PMC
# passes (each counter group its own run, no tracing domains) for the bench kernels at the bench
# mesh (64^2, P=8) and the HBM-regime mesh (1024^2, P=8), plus the FETCH_SIZE calibration run
# (sem_dss reads exactly ne^2*81*8 bytes with 8-byte loads, the access width of the apply kernels).
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
echo bench ok; cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python bench.py --cpu-seconds 0 > $OUT/trace.log 2>&1 || { echo trace failed; tail $OUT/trace.log; exit 1; }
echo trace ok
i=0
for PMC in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PMC -d $OUT/pmc$i -o pmc --output-format csv -- python tools/kbench.py --meshes 8:64,8:1024 --reps 50 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; }
done
for PMC in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $PMC -d $OUT/cal_$PMC -o pmc --output-format csv -- python tools/kbench.py --dss 1024 > $OUT/cal_$PMC.log 2>&1 || { echo "calibration $PMC failed"; tail -3 $OUT/cal_$PMC.log; }
done
echo done
