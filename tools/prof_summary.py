"""Summarise a tools/gpu_bench_prof.sh (or gpu_prof.sh) output directory.

Kernel durations come from the per-dispatch kernel trace, grouped by (kernel, grid size), so a
kernel launched at two mesh sizes (the bench mesh and the HBM-regime mesh) is reported per size;
counters are per-dispatch means over the PMC passes, grouped the same way.

python tools/prof_summary.py gpurun_out/<tag> [kernel-substring]
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    kfilter = sys.argv[2] if len(sys.argv) > 2 else "sem::"
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if kfilter not in name:
                continue
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
            durs[(name[:60], grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print("kernel trace (per dispatch, grouped by grid size):")
    for (name, grid), v in sorted(durs.items()):
        print(f"  {name:60s} grid={grid:>9s} calls={len(v):5d} avg={statistics.mean(v) / 1e3:9.2f}us "
              f"median={statistics.median(v) / 1e3:9.2f}us min={min(v) / 1e3:9.2f}us")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv")) +
                    glob.glob(os.path.join(d, "cal_*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kfilter not in r["Kernel_Name"] and "dss_kernel" not in r["Kernel_Name"]:
                continue
            n = int(r.get("Dispatches") or 1)   # tools/pmc_compact.py rows: a mean over n dispatches
            agg[(r["Kernel_Name"][:60], r["Grid_Size"])][r["Counter_Name"]].append((float(r["Counter_Value"]), n))
    print("counters (per-dispatch means):")
    for (name, grid), cs in sorted(agg.items()):
        print(f"  {name}  grid={grid}")
        for c, v in sorted(cs.items()):
            n = sum(k for _, k in v)
            print(f"     {c:28s} {sum(x * k for x, k in v) / n:18.1f}   (n={n})")


if __name__ == "__main__":
    main()
