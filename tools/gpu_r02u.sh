#!/bin/bash
# Kernel-level breakdown of the NS velocity solve and Schur matvec at the cfg4 mesh (48^2, P=8).
set -o pipefail
O=gpurun_out/r02u; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python -u tools/velocity_bench.py --ne 48 --P 8 --configs nested:cr --reps 20 > $O/vb48.log 2>&1 || { tail -5 $O/vb48.log; exit 1; }
tail -2 $O/vb48.log | cut -c1-1500
head -25 $O/trace/trace_kernel_stats.csv | cut -c1-250
