"""HBM traffic per launch from tools/pmc_run.sh passes -> profiles/pmc_traffic.json (read by bench.py).

FETCH_SIZE / WRITE_SIZE are the L2's memory-side request counters (MI355X_MICROARCH.md, HBM section):
WRITE_SIZE counts the bytes of our 8-byte-per-lane stores exactly, FETCH_SIZE under-reports reads by
an access-width-dependent factor, so it is calibrated on a kernel of the same access width with a known
byte count (sem_dss: 8-byte loads, reads exactly ne^2 (P+1)^2 8 bytes; tools/kbench.py --dss NE).
Each workload's entry is keyed by the workload name bench.py prints and records the exact kernel
instantiation it was measured on; bench.py uses it only when that name matches the kernel it runs.

python tools/pmc_traffic.py --cal DIR:NE --workload NAME=DIR:ALGO_BYTES [...] [--out profiles/pmc_traffic.json]
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_dispatch(d, counter, kfilter):
    """{kernel name: mean per-dispatch value of `counter`} over the pmc passes under d (units as reported)."""
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kfilter in r["Kernel_Name"]:
                # a tools/pmc_compact.py row is already a mean over `Dispatches` dispatches
                acc[r["Kernel_Name"]].append((float(r["Counter_Value"]), int(r.get("Dispatches") or 1)))
    return {k: (sum(x * n for x, n in v) / sum(n for _, n in v), sum(n for _, n in v)) for k, v in acc.items()}


def short(name):
    name = name.replace("void ", "")
    return name[:name.index("(")] if "(" in name else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cal", required=True, help="DIR:NE of a kbench --dss NE run (P = 8)")
    ap.add_argument("--workload", action="append", default=[], help="NAME=DIR:ALGORITHMIC_BYTES")
    ap.add_argument("--kernel", default="sem::", help="kernel-name filter")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    cdir, ne = a.cal.rsplit(":", 1)
    ne = int(ne)
    f = per_dispatch(cdir, "FETCH_SIZE", "dss_kernel")
    (fk, (fv, _)), = f.items()
    true_read = ne * ne * 81 * 8
    corr = true_read / (fv * 1024.0)
    out = {"_doc": __doc__.split("\n\n")[1].replace("\n", " "), "round": a.tag, "fetch_correction": corr,
           "calibration": {"kernel": short(fk), "read_bytes": true_read, "fetch_size_kb": fv}, "workloads": {}}
    for w in a.workload:
        name, rest = w.split("=", 1)
        d, algo = rest.rsplit(":", 1)
        fs, ws = per_dispatch(d, "FETCH_SIZE", a.kernel), per_dispatch(d, "WRITE_SIZE", a.kernel)
        k = max(fs, key=lambda n: fs[n][1] * fs[n][0])     # the dominant kernel of the run
        hbm = fs[k][0] * 1024.0 * corr + ws[k][0] * 1024.0
        out["workloads"][name] = {"kernel": short(k), "dispatches": fs[k][1], "fetch_size_kb": fs[k][0],
                                  "write_size_kb": ws[k][0], "hbm_bytes_per_launch": hbm,
                                  "algorithmic_bytes_per_launch": float(algo),
                                  "traffic_over_algorithmic": hbm / float(algo), "source": d}
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
