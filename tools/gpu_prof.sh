#!/bin/bash
# rocprofv3: kernel trace + stats, then PMC counter passes (each its own run, no tracing domains).
set -o pipefail
TAG=${1:-prof}
shift
ARGS=${KB_ARGS:-"--meshes 8:64,8:1024 --reps 50 --algo 2"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
R="timeout -k 10 300 rocprofv3"
$R --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python tools/kbench.py $ARGS > $OUT/trace.log 2>&1 || { echo trace failed; tail $OUT/trace.log; exit 1; }
echo trace ok
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  $R --pmc $PMC -d $OUT/pmc$i -o pmc --output-format csv -- python tools/kbench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; }
done
find $OUT -name "*.csv" | head -20
