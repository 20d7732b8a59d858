#!/bin/bash
# rocprofv3 evidence for one command: a kernel trace with --stats, then one --pmc pass per counter
# group, each in a run of its own (no tracing domains next to --pmc; at most 8 SQ, 4 TCC counters a
# pass; FETCH_SIZE and WRITE_SIZE in separate passes).  Summarise with tools/prof_summary.py OUTDIR.
#   tools/pmc_run.sh OUTDIR -- python tools/kbench.py --meshes 8:64 --reps 50
set -o pipefail
OUT=$1; shift; [ "$1" = "--" ] && shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- "$@" \
  > "$OUT/trace.log" 2>&1 || { echo "trace failed: $OUT"; tail -5 "$OUT/trace.log"; exit 1; }
i=0
for PMC in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
    "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
    "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PMC -d "$OUT/pmc$i" -o pmc --output-format csv -- "$@" > "$OUT/pmc$i.log" 2>&1 \
    || { echo "pmc pass $i failed: $OUT"; tail -3 "$OUT/pmc$i.log"; exit 1; }
done
python tools/pmc_compact.py "$OUT" && python tools/prof_summary.py "$OUT" > "$OUT/prof_summary.txt" 2>&1
echo "pmc ok: $OUT"
