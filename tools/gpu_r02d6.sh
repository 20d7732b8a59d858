#!/bin/bash
# Diagnostic: one-shot vs column-chunked condensed CD solve at 32^2 / 64^2, P = 12 and 128^2, P = 8.
set -o pipefail
O=gpurun_out/r02d6; mkdir -p $O
timeout -k 10 200 python -u tools/chunk_probe.py --ne 32 --P 12 > $O/p32.log 2>&1 || { tail -3 $O/p32.log; exit 1; }
grep "^{" $O/p32.log
timeout -k 10 300 python -u tools/chunk_probe.py --ne 64 --P 12 --chunks 0,6,16 > $O/p64.log 2>&1 || { tail -3 $O/p64.log; exit 1; }
grep "^{" $O/p64.log
timeout -k 10 300 python -u tools/chunk_probe.py --ne 128 --P 8 --chunks 0,6 > $O/p128.log 2>&1 || { tail -3 $O/p128.log; exit 1; }
grep "^{" $O/p128.log
