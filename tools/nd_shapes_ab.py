"""A/B of sem_front_gemv's launch shapes on one factor (cfg5 velocity Jacobian of tools/nd_probe.py's smooth
linearisation): for each policy the plan is rebuilt and captured, the graph-replayed solve timed (median of
--solves, the policies alternated --rounds times) and every step timed eagerly; the solutions must agree to
rounding.  Policies: "default" (NestedDissectionSolver._launch_shape), "wide64" (64 lanes always with 16 rows
per workgroup), "narrow64" (64 lanes always with 4 rows), "lanes32" (rows of >= 1024 doubles on 32 lanes),
"wide256" (the wide tile whenever it gives >= 256 workgroups), "fit" (the narrow tile when the wide one pads the rows by > 15 % more), "colsN" (the column form for forward front levels
of median row length <= N; the default is 64).

python tools/nd_shapes_ab.py [--ne 128 --P 12 --solves 30 --rounds 2 --out FILE]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=128)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--solves", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--policies", default="default,wide64,narrow64,lanes32,wide256")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    from sem_amd.solvers.nested_dissection import NestedDissectionSolver as ND
    import ctypes as C
    from sem_amd import _lib
    dev = torch.device("cuda", 0)
    ns = NavierStokesSolver(1.0, 1.0, 1e3, 1e6 / 0.71, args.P, args.ne, args.ne, mtol=1e-10, mtol_newton=1e-10,
                            iprint=[], velocity_graph=False)
    x, y = ns.points
    u0 = 1e-2 * np.sin(np.pi * x) * np.sin(2 * np.pi * y)
    v0 = -1e-2 * np.sin(2 * np.pi * x) * np.sin(np.pi * y)
    ns._get_residuals(u0, v0, np.zeros(ns.N), 0.5 - x)
    ns._calc_jacobians(u0, v0)
    nd = ns._velocity_solver()
    assert nd.interior == "nd"
    r = np.random.default_rng(5)
    bu, bv = (ns._dev(r.uniform(-1, 1, ns.N)) for _ in range(2))
    base_shape = ND._launch_shape.__func__

    def shape_for(policy):
        def f(cls, K, R):
            kp = int(np.median(K)) // 2
            if policy == "wide64" and kp >= 96:
                return 64, 16
            if policy == "narrow64" and kp >= 96:
                return 64, 4
            if policy == "wide256":      # the wide tile from 256 workgroups on (default: 2048)
                lanes, _ = base_shape(cls, K, R)
                wide, narrow = cls.SHAPES[lanes]
                return lanes, wide if int(((R + wide - 1) // wide).sum()) >= 256 else narrow
            if policy == "fit":          # the narrow tile when the wide one pads the fronts' rows by > 15 % more
                lanes, rows = base_shape(cls, K, R)
                wide, narrow = cls.SHAPES[lanes]
                tw, tn = int(((R + wide - 1) // wide).sum()), int(((R + narrow - 1) // narrow).sum())
                if rows == wide and R.sum() / (tn * narrow) > 1.15 * R.sum() / (tw * wide):
                    return lanes, narrow
                return lanes, rows
            if policy == "lanes32" and kp >= 512:
                wide, narrow = cls.SHAPES[32]
                return 32, wide if int(((R + wide - 1) // wide).sum()) >= 2048 else narrow
            return base_shape(cls, K, R)
        return classmethod(f)

    lib = _lib.load()
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    res, ref = {}, None
    policies = args.policies.split(",")
    base_form = ND._launch_form
    for _ in range(args.rounds):
        for pol in policies:
            ND._launch_shape = shape_for(pol)
            if pol.startswith("cols"):     # the column form for forward front levels up to this median row length
                lim = int(pol[4:])
                ND._launch_form = lambda self, back, nf, K, leaves, lim=lim: (
                    0 if leaves or back else int(int(np.median(K)) <= lim))
            else:
                ND._launch_form = base_form
            nd._hip = nd._hip_plan()
            nd.capture()
            for _ in range(3):
                nd.solve(bu, bv)
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(args.solves):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                xu, xv = nd.solve(bu, bv)
                b.record()
                torch.cuda.synchronize(dev)
                ts.append(a.elapsed_time(b))
            if ref is None:
                ref = (xu.clone(), xv.clone())
            diff = float(max((xu - ref[0]).abs().max(), (xv - ref[1]).abs().max()) / ref[0].abs().max())
            W = torch.stack((bu.view(nd.NX, -1), bv.view(nd.NX, -1)), 1).reshape(-1).clone()
            ev = []
            for entry in nd._hip:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                nd._launch(lib, entry, W, st)
                b.record()
                ev.append((a, b, entry[0]))
            torch.cuda.synchronize(dev)
            steps = [{"us": a.elapsed_time(b) * 1e3, "lanes": getattr(d, "lanes", None), "rows": getattr(d, "rows", None)}
                     for a, b, d in ev]
            e = res.setdefault(pol, {"solve_ms": [], "steps_us": [], "rel_diff": 0.0})
            e["solve_ms"].append(float(np.median(ts)))
            e["steps_us"].append([s["us"] for s in steps])
            e["shapes"] = [(s["lanes"], s["rows"]) for s in steps]
            e["rel_diff"] = max(e["rel_diff"], diff)
    out = {"config": f"velocity solve {args.ne}x{args.ne} P={args.P}", "policies": {}}
    for pol, e in res.items():
        out["policies"][pol] = {"solve_ms": e["solve_ms"], "steps_us_median": np.median(np.array(e["steps_us"]),
                                                                                        axis=0).round(1).tolist(),
                                "shapes": e["shapes"], "rel_diff": e["rel_diff"]}
    print(json.dumps({p: (v["solve_ms"], v["rel_diff"]) for p, v in out["policies"].items()}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
