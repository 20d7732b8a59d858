"""Velocity-Jacobian device solve timings (sem_amd/solvers/velocity_solve.py): factorisation and
solve per configuration (interior elimination x interface sweep, eager vs hipGraph) at a smooth
linearisation state, with the solve's residual checked through the matrix-free Jacobian, and the
Schur-complement matvec of _get_update (eager vs one captured graph).

python tools/velocity_bench.py --ne 32 --P 8 --Re 1000
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
    ap.add_argument("--ne", type=int, default=32)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--Re", type=float, default=1000.0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--configs", default="nested:cr,nested:thomas", help="interior:sweep,...")
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    from sem_amd.solvers.velocity_solve import VelocityJacobianSolver
    out = {"mesh": f"{args.ne}x{args.ne}", "P": args.P, "Re": args.Re}
    from sem_amd.solvers.navier_stokes import _SchurComplement
    for cfg in args.configs.split(","):
        interior, sweep = cfg.split(":")
        ns = NavierStokesSolver(1.0, 1.0, args.Re, 0.0, args.P, args.ne, args.ne, u_N=1.0, iprint=[],
                                velocity_interior=interior, velocity_sweep=sweep, velocity_graph=False)
        x, y = ns.points
        u = np.sin(np.pi * x) * np.sin(np.pi * y) * (y ** 2)
        v = -np.sin(np.pi * x) * np.sin(2 * np.pi * y) * 0.3
        ns._get_residuals(u, v, np.zeros(ns.N), np.zeros(ns.N))
        ns._calc_jacobians(u, v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vs = ns._velocity_solver()
        torch.cuda.synchronize()
        t_factor = time.perf_counter() - t0
        r = np.random.default_rng(1)
        bu, bv = ns._dev(r.uniform(-1, 1, ns.N)), ns._dev(r.uniform(-1, 1, ns.N))
        res = {}
        for mode in ("eager", "graph"):
            if mode == "graph":
                t0 = time.perf_counter()
                ok = vs.capture()
                torch.cuda.synchronize()
                res["capture_s"] = time.perf_counter() - t0
                if not ok:
                    res["graph"] = "capture refused"
                    continue
            xu, xv = vs.solve(bu, bv)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                xu, xv = vs.solve(bu, bv)
            torch.cuda.synchronize()
            res[f"{mode}_solve_ms"] = (time.perf_counter() - t0) / args.reps * 1e3
            # J x = b through the matrix-free Jacobian (Dirichlet rows: identity)
            Z = torch.zeros(ns.N, dtype=torch.float64, device=bu.device)
            ru, rv, _ = ns._get_dresiduals(xu, xv, Z)
            res[f"{mode}_rel_residual"] = max((ru - bu).abs().max().item(), (rv - bv).abs().max().item()) / max(
                xu.abs().max().item(), xv.abs().max().item())
        res["factor_s"] = t_factor
        # the Schur-complement matvec of _get_update: eager, and captured whole in one graph
        dp = ns._dev(r.uniform(-1, 1, ns.N))
        for graph in (False, True):
            S = _SchurComplement(ns, vs, graph=graph)
            y0 = S(dp)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                y = S(dp)
            torch.cuda.synchronize()
            res[f"schur_{'graph' if graph else 'eager'}_ms"] = (time.perf_counter() - t0) / args.reps * 1e3
            if graph:
                res["schur_graph_vs_eager"] = (y - y0).abs().max().item() / y0.abs().max().item()
        res["mem_GB"] = torch.cuda.max_memory_allocated() / 1e9
        out[cfg] = res
        print(json.dumps({cfg: res}), flush=True)
        del vs, ns
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
