"""The nested-dissection velocity solve (sem_amd/solvers/nested_dissection.py) against the line condensation
(velocity_solve.py) on one linearisation: factor times, resident memory, graph-replayed solve times (HIP events,
median of --solves), the two solutions' difference, both factors' backward-error probes, and the ND solve's
per-step device time (eager, events around each launch pair) with each step's operator bytes.

python tools/nd_probe.py [--ne 128 --P 12 --Ra 1e6 --solves 20 --lines 1 --out FILE]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=128)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--Ra", type=float, default=1e6)
    ap.add_argument("--solves", type=int, default=20)
    ap.add_argument("--lines", type=int, default=1, help="also factor and time the line condensation")
    ap.add_argument("--steps", type=int, default=1, help="per-step eager timing of the ND solve")
    ap.add_argument("--ab-forms", type=int, default=0,
                    help="also time every launch in sem_front_gemv's form 0 (forms='rows') against the default plan")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    from sem_amd.solvers.nested_dissection import NestedDissectionSolver
    import ctypes as C
    from sem_amd import _lib
    Re, Pr = 1e3, 0.71
    dev = torch.device("cuda", 0)
    ns = NavierStokesSolver(1.0, 1.0, Re, args.Ra / Pr, args.P, args.ne, args.ne, mtol=1e-10, mtol_newton=1e-10,
                            iprint=[])
    N = ns.N
    x, y = ns.points
    u0 = 1e-2 * np.sin(np.pi * x) * np.sin(2 * np.pi * y)
    v0 = -1e-2 * np.sin(2 * np.pi * x) * np.sin(np.pi * y)
    ns._get_residuals(u0, v0, np.zeros(N), 0.5 - x)
    ns._calc_jacobians(u0, v0)
    out = {"config": f"velocity solve {args.ne}x{args.ne} P={args.P}", "N": N}
    r = np.random.default_rng(5)
    bu, bv = (ns._dev(r.uniform(-1, 1, N)) for _ in range(2))

    def timed(vs):
        for _ in range(3):
            vs.solve(bu, bv)
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(args.solves):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            xu, xv = vs.solve(bu, bv)
            b.record()
            torch.cuda.synchronize(dev)
            ts.append(a.elapsed_time(b))
        return ts, xu, xv

    def relres(xu, xv):
        ju, jv, _ = ns._get_dresiduals(xu, xv, torch.zeros_like(xu))
        return float(max((ju - bu).abs().max(), (jv - bv).abs().max()) / max(bu.abs().max(), bv.abs().max()))

    torch.cuda.synchronize(dev)
    m0 = torch.cuda.memory_allocated(dev)
    t0 = time.perf_counter()
    nd = NestedDissectionSolver(args.P, args.ne, args.ne, dev)
    t_tree = time.perf_counter() - t0
    nd.profile = True
    nd.factor_mesh(ns._mesh, dir_mask=ns._dir.mask, dir_sides=ns._dir.sides, **ns._jac_kw)
    torch.cuda.synchronize(dev)
    t_f = time.perf_counter() - t0
    nd.set_operator(ns._velocity_apply_lines)
    eta = nd.check_refinement()
    cap = nd.capture()
    torch.cuda.synchronize(dev)
    out["nd"] = {"tree_s": t_tree, "factor_s": t_f, "phases": nd.timing, "resident_GB": (torch.cuda.memory_allocated(dev)
                 - m0) / 1e9, "bytes_per_solve": nd.bytes_per_solve(), "eta": eta, "refine": nd.refine,
                 "graph": cap, "fronts": len(nd.tree.fronts), "depth": nd.tree.depth, "launches": len(nd._hip),
                 "split": nd.split, "split_eta": nd.split_eta}
    ts, xu, xv = timed(nd)
    med = float(np.median(ts))
    out["nd"].update({"solve_ms_median": med, "solve_ms_min": float(min(ts)), "rel_residual": relres(xu, xv),
                      "frac_8TBs": nd.bytes_per_solve() / (med * 1e-3) / 8e12})
    # bitwise: graph replay against the eager solve
    xe = nd._solve_lines(torch.stack((bu.view(nd.NX, -1), bv.view(nd.NX, -1)), 1).reshape(nd.NX, -1))
    out["nd"]["graph_equals_eager"] = bool(torch.equal(xe.view(nd.NX, 2, -1)[:, 0].reshape(-1), xu)
                                           and torch.equal(xe.view(nd.NX, 2, -1)[:, 1].reshape(-1), xv))
    if args.ab_forms:   # the same factor, every launch in form 0, then back to the default plan (alternated)
        ts_auto, ts_rows = [], []
        for _ in range(3):
            for forms, acc in (("rows", ts_rows), ("auto", ts_auto)):
                nd.forms = forms
                nd._hip = nd._hip_plan()
                nd.capture()
                t_, xu_f, xv_f = timed(nd)
                acc.extend(t_)
                if forms == "rows":
                    xr = (xu_f.clone(), xv_f.clone())
        out["nd"]["ab_forms"] = {"rows_ms_median": float(np.median(ts_rows)), "auto_ms_median": float(np.median(ts_auto)),
                                 "rel_diff": float(max((xu_f - xr[0]).abs().max(), (xv_f - xr[1]).abs().max())
                                                   / max(xr[0].abs().max(), xr[1].abs().max()))}
    if args.steps:
        lib = _lib.load()
        W = torch.stack((bu.view(nd.NX, -1), bv.view(nd.NX, -1)), 1).reshape(-1).clone()
        st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        per = []
        for rep in range(3):
            rows = []
            for entry in nd._hip:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                nd._launch(lib, entry, W, st)
                b.record()
                rows.append((a, b, entry[0]))
            torch.cuda.synchronize(dev)
            per.append([a.elapsed_time(b) * 1e3 for a, b, _ in rows])
        us = np.median(np.array(per), axis=0)
        steps = []
        for k, (d, keep, sc, sp) in enumerate(nd._hip):
            if isinstance(d, _lib.SemLeafLaunch):     # the split leaves: one workgroup per element
                byts = nd._leafB.numel() * 8
                steps.append({"step": k, "back": 0, "leaf": "split", "fronts": d.nelem, "tiles": d.nelem,
                              "us": float(us[k]), "op_MB": byts / 1e6, "TBs": byts / (us[k] * 1e-6) / 1e12})
                continue
            dims = keep["dims"].cpu().numpy()
            byts = int((dims[:, 0].astype(np.int64) * dims[:, 1]).sum() * 8) + (sp["coef"].numel() * 8 if sp else 0)
            steps.append({"step": k, "back": d.back, "fronts": int(dims.shape[0]), "tiles": d.ntiles, "rows": d.rows,
                          "lanes": d.lanes, "form": d.form,
                          "us": float(us[k]), "op_MB": byts / 1e6, "TBs": byts / (us[k] * 1e-6) / 1e12})
        out["nd"]["steps"] = steps
        out["nd"]["steps_sum_us"] = float(us.sum())
    if args.lines:
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ns._velocity_interior, ns._velo = "nested", None     # the line condensation (the default is now ND)
        vs = ns._velocity_solver()
        torch.cuda.synchronize(dev)
        out["lines"] = {"factor_s": time.perf_counter() - t0, "eta": vs.refine_eta}
        ts, lu, lv = timed(vs)
        out["lines"].update({"solve_ms_median": float(np.median(ts)), "rel_residual": relres(lu, lv)})
        out["nd_vs_lines_rel_diff"] = float(max((xu - lu).abs().max(), (xv - lv).abs().max())
                                            / max(lu.abs().max(), lv.abs().max()))
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
