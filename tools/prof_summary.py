"""Summarise a tools/gpu_prof.sh output directory: kernel stats + per-dispatch counter means."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
kfilter = sys.argv[2] if len(sys.argv) > 2 else "apply_tp"
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if kfilter in r["Name"]:
            print(f"{r['Name'][:60]:60s} calls={r['Calls']} avg={float(r['AverageNs'])/1e3:.2f}us "
                  f"min={float(r['MinNs'])/1e3:.2f}us max={float(r['MaxNs'])/1e3:.2f}us")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if kfilter not in r["Kernel_Name"]:
            continue
        agg[(r["Kernel_Name"][:40], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
