"""Shrink a tools/pmc_run.sh output directory in place, so that it travels back from the GPU box
(gpurun copies at most 64 MiB of gpurun_out/): every *counter_collection.csv becomes one row per
(kernel, grid, counter) holding the per-dispatch mean and the dispatch count, and every
*kernel_trace.csv keeps only the columns tools/prof_summary.py reads.
tools/prof_summary.py and tools/pmc_traffic.py read both forms.

python tools/pmc_compact.py OUTDIR
"""
import collections
import csv
import glob
import os
import sys


def compact_counters(f):
    acc = collections.defaultdict(list)
    with open(f) as fh:
        for r in csv.DictReader(fh):
            n = int(r.get("Dispatches") or 1)
            acc[(r["Kernel_Name"], r["Grid_Size"], r["Counter_Name"])].append((float(r["Counter_Value"]), n))
    with open(f, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value", "Dispatches"])
        for (k, g, c), v in sorted(acc.items()):
            n = sum(x[1] for x in v)
            w.writerow([k, g, c, sum(x[0] * x[1] for x in v) / n, n])


def compact_trace(f):
    keep = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
            keep.append((r["Kernel_Name"], grid, r["Start_Timestamp"], r["End_Timestamp"]))
    with open(f, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Grid_Size", "Start_Timestamp", "End_Timestamp"])
        w.writerows(keep)


def main():
    d = sys.argv[1]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        compact_counters(f)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        compact_trace(f)
    for f in glob.glob(os.path.join(d, "**", "*"), recursive=True):   # other rocprofv3 outputs
        if os.path.isfile(f) and not f.endswith((".csv", ".log", ".txt")) and os.path.getsize(f) > (1 << 20):
            os.remove(f)


if __name__ == "__main__":
    main()
