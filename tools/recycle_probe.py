"""Recycled-Krylov probe on the device solvers: repeated _get_update calls with one linearisation
(the Boussinesq block-Jacobi pattern), consistent right-hand sides, iterations and times per call."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from sem_amd.solvers import ConvectionDiffusionSolver, NavierStokesSolver
    ne = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rng = np.random.default_rng(0)
    ns = NavierStokesSolver(1.0, 1.0, 1e3, 1e3 / 0.71, 8, ne, ne, mtol=1e-13, mtol_newton=1e-13, iprint=[])
    x, y = ns.points
    u = 0.01 * np.sin(np.pi * x) * np.sin(np.pi * y)
    v = -0.01 * np.sin(2 * np.pi * x) * np.sin(np.pi * y)
    p = np.zeros(ns.N)
    ns._get_residuals(u, v, p, 0.5 - x)
    ns._calc_jacobians(u, v)
    for k in range(8):
        du, dv, dp = (rng.uniform(-1, 1, ns.N) for _ in range(3))
        ru, rv, rc = ns._get_dresiduals(du, dv, dp)
        t0 = time.perf_counter()
        ns._get_update(ru, rv, rc, du0=np.zeros(ns.N), dv0=np.zeros(ns.N), dp0=np.zeros(ns.N))
        torch.cuda.synchronize()
        rcy = ns._schur_recycle
        print(f"NS call {k}: {ns.schur_matvecs} Schur matvecs, {time.perf_counter() - t0:.3f} s, recycle k={rcy.k}",
              flush=True)
    cd = ConvectionDiffusionSolver(1.0, 1.0, 710.0, 8, ne, ne, T_W=0.5, T_E=-0.5, mtol=1e-13)
    cd._get_residuals(np.zeros(cd.N), u, v)
    for k in range(8):
        b = cd._get_dresiduals(rng.uniform(-1, 1, cd.N))
        t0 = time.perf_counter()
        cd._get_update(b, dT0=np.zeros(cd.N))
        torch.cuda.synchronize()
        print(f"CD call {k}: {cd.matvecs} matvecs, {time.perf_counter() - t0:.3f} s, recycle k={cd._recycle.k}",
              flush=True)


if __name__ == "__main__":
    main()
