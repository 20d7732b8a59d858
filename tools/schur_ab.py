"""A/B of the Schur-complement preconditioner on cfg4's block solves.

At the committed converged Ra = 1e6 state (tests/golden/cfg4_state.npz: 48^2 elements, P = 8), linearise the
device NS solver and run one NS block-Jacobi solve (_get_update, NavierStokes_Solver.py:162-236) per
preconditioner with the couplers' mtol_internal = 1e-13 and the reference's stopping rule
||r||_2 <= mtol sqrt(N).  Right-hand side: the device Jacobian applied to a smooth step (a consistent
right-hand side, as the cfg4 GPU test uses).  Reports Schur matvecs, wall time, the time of the matvecs alone
(matvecs x one graph-replayed Schur matvec) and so the Krylov-basis share, and the velocity error of the update.

python tools/schur_ab.py [--precond mass,pcd] [--out file.jsonl]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precond", default="mass,pcd")
    ap.add_argument("--mtol", type=float, default=1e-13)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    NE, P, RE, RA, PR = 48, 8, 1e3, 1e6, 0.71
    x = np.load(os.path.join(ROOT, "tests", "golden", "cfg4_state.npz"))["x"]
    N = (NE * P + 1) ** 2
    T, u, v, p = x[:N], x[N:2 * N], x[2 * N:3 * N], x[3 * N:]
    dev = torch.device("cuda", 0)
    lines = []
    for pc in a.precond.split(","):
        ns = NavierStokesSolver(1.0, 1.0, RE, RA / PR, P, NE, NE, mtol=a.mtol, mtol_newton=a.mtol, iprint=[],
                                schur_precond=pc)
        X, Y = ns.points
        ns._get_residuals(u, v, p, T)
        ns._calc_jacobians(u, v)
        step = (1e-3 * np.sin(np.pi * X) * np.sin(2 * np.pi * Y), -2e-3 * np.sin(2 * np.pi * X) * np.sin(np.pi * Y),
                1e-2 * np.cos(np.pi * X) * np.cos(np.pi * Y))
        rhs = [ns._dev(r) for r in ns._get_dresiduals(*(ns._dev(s) for s in step))]
        z = torch.zeros(N, dtype=torch.float64, device=dev)
        t0 = time.perf_counter()
        ns._get_update(*rhs, du0=z, dv0=z, dp0=z)          # factor + graph capture + a first solve
        torch.cuda.synchronize(dev)
        first = time.perf_counter() - t0
        t0 = time.perf_counter()
        du, dv, dp = ns._get_update(*rhs, du0=z, dv0=z, dp0=z)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        nmv = ns.schur_matvecs
        # one Schur matvec (graph replay), and its preconditioner, timed alone
        sch = ns._schur
        q = torch.rand(N, dtype=torch.float64, device=dev)
        for _ in range(3):
            sch(q)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            sch(q)
        e1.record()
        torch.cuda.synchronize(dev)
        mv_ms = e0.elapsed_time(e1) / 20
        pc_ms = 0.0
        if pc == "pcd":
            e0.record()
            for _ in range(20):
                ns._pcd(q)
            e1.record()
            torch.cuda.synchronize(dev)
            pc_ms = e0.elapsed_time(e1) / 20
        lin = ns._get_dresiduals(du, dv, dp)
        res = float(np.sqrt(sum(float(((s - r) ** 2).sum()) for s, r in zip(lin, rhs))))
        verr = max(float((du - ns._dev(step[0])).abs().max()) / np.abs(step[0]).max(),
                   float((dv - ns._dev(step[1])).abs().max()) / np.abs(step[1]).max())
        out = {"config": "cfg4 NS block solve at cfg4_state (48^2, P=8, Ra=1e6)", "precond": pc, "N": N,
               "schur_matvecs": nmv, "wall_s": wall, "first_call_s": first, "schur_matvec_ms": mv_ms,
               "precond_ms": pc_ms, "matvec_time_s": nmv * (mv_ms + pc_ms) / 1e3,
               "krylov_share": 1.0 - nmv * (mv_ms + pc_ms) / 1e3 / wall, "residual": res,
               "tolerance": a.mtol * np.sqrt(N), "velocity_rel_err": verr}
        print(json.dumps(out), flush=True)
        lines.append(out)
        del ns
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for l in lines:
                f.write(json.dumps(l) + "\n")


if __name__ == "__main__":
    main()
