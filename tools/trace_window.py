"""Per-kernel breakdown of the last `reps` repetitions of an operation in a rocprofv3 kernel trace.

The window starts at the (2 reps)-th last dispatch of a marker kernel that runs `per_rep` times per
repetition (default: sem::ns_apply_kernel, twice per Schur-complement matvec).

python tools/trace_window.py <trace_kernel_trace.csv | rocprofv3 -d dir> [reps] [marker] [per_rep] [--save out.csv]
(--save: the window's dispatches as a small CSV, so the full trace need not travel back from the GPU box)
"""
import collections
import csv
import glob
import os
import sys


def main():
    save = None
    if "--save" in sys.argv:
        i = sys.argv.index("--save")
        save = sys.argv[i + 1]
        del sys.argv[i:i + 2]
    path = sys.argv[1]
    if os.path.isdir(path):   # a rocprofv3 -d directory: its kernel trace
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    marker = sys.argv[3] if len(sys.argv) > 3 else "ns_apply"
    per_rep = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    seg = rows[idx[-reps * per_rep]:]
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = r["Kernel_Name"][:80] + " grid=%s,%s" % (r["Grid_Size_X"], r["Grid_Size_Y"])
        tot[k][0] += 1
        tot[k][1] += d
    if save:
        with open(save, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Kernel_Name", "Grid_Size_X", "Grid_Size_Y", "Start_Timestamp", "End_Timestamp"])
            for r in seg:
                w.writerow([r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"], r["Start_Timestamp"],
                            r["End_Timestamp"]])
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in tot.values())
    print(f"per repetition: span {span / reps:.1f} us, kernel busy {busy / reps:.1f} us, {len(seg) / reps:.1f} launches")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{v[1] / reps:8.1f} us  x{v[0] / reps:4.1f}  {k}")


if __name__ == "__main__":
    main()
