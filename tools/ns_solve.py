"""Lid-driven cavity Navier-Stokes solve on the device (cfg3: Re = 1000, 32 x 32 elements, P = 8;
Examples/NavierStokes_Example.py:20-36 at BASELINE.json's configuration).

python tools/ns_solve.py --ne 32 --P 8 --Re 1000 [--out result.json]
Prints per-Newton residual norms and Schur-complement matvec counts, the velocity-factorisation
and total wall times, and the solution checksums (norms, strided samples) that
tests/golden/cfg3_checksums.npz pins.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


# Ghia, Ghia & Shin (1982), J. Comput. Phys. 48:387, Tables I-II, Re = 1000: u on the vertical centre
# line x = 1/2 and v on the horizontal centre line y = 1/2 (the benchmark the reference's example
# names, Examples/NavierStokes_Example.py:15)
GHIA_RE1000_U = [(0.9766, 0.65928), (0.9688, 0.57492), (0.9609, 0.51117), (0.9531, 0.46604), (0.8516, 0.33304),
                 (0.7344, 0.18719), (0.6172, 0.05702), (0.5000, -0.06080), (0.4531, -0.10648), (0.2813, -0.27805),
                 (0.1719, -0.38289), (0.1016, -0.29730), (0.0703, -0.22220), (0.0625, -0.20196), (0.0547, -0.18109)]
GHIA_RE1000_V = [(0.9688, -0.21388), (0.9609, -0.27669), (0.9531, -0.33714), (0.9453, -0.39188), (0.9063, -0.51550),
                 (0.8594, -0.42665), (0.8047, -0.31966), (0.5000, 0.02526), (0.2344, 0.32235), (0.2266, 0.33075),
                 (0.1563, 0.37095), (0.0938, 0.32627), (0.0781, 0.30353), (0.0703, 0.29012), (0.0625, 0.27485)]


def ghia_deviation(ns, u, v):
    """Largest |ours - Ghia| over the Re = 1000 centre-line points (interpolated with _get_interpol)."""
    yu = np.array([a for a, _ in GHIA_RE1000_U])
    xv = np.array([a for a, _ in GHIA_RE1000_V])
    up = np.asarray(ns._get_interpol(u, (np.full((1, yu.size), 0.5), yu[None, :]))).ravel()
    vp = np.asarray(ns._get_interpol(v, (xv[:, None], np.full((xv.size, 1), 0.5)))).ravel()
    du = np.abs(up - np.array([b for _, b in GHIA_RE1000_U])).max()
    dv = np.abs(vp - np.array([b for _, b in GHIA_RE1000_V])).max()
    return float(du), float(dv), up.tolist(), vp.tolist()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=32)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--Re", type=float, default=1000.0)
    ap.add_argument("--mtol", type=float, default=1e-7)
    ap.add_argument("--mtol-newton", type=float, default=1e-5)
    ap.add_argument("--out", default="")
    ap.add_argument("--schur-precond", default="mass", choices=["pcd", "mass"])
    ap.add_argument("--continuation", default="",
                    help="comma-separated Reynolds numbers solved first, each from the previous solution "
                         "(_get_solution's u0, v0, p0), e.g. 100,400")
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    res = [float(r) for r in args.continuation.split(",") if r] + [args.Re]
    u = v = p = None
    stages = []
    t_all = time.perf_counter()
    for Re in res:
        t0 = time.perf_counter()
        ns = NavierStokesSolver(1.0, 1.0, Re, 0.0, args.P, args.ne, args.ne, u_N=1.0, mtol=args.mtol,
                                mtol_newton=args.mtol_newton, iprint=["NEWTON_iter", "NEWTON_suc", "LU_suc"],
                                schur_precond=args.schur_precond)
        ns._progress = 200    # print the Schur GMRES estimate every 200 iterations
        t_setup = time.perf_counter() - t0
        T = np.zeros(ns.N)
        t0 = time.perf_counter()
        u, v, p = ns._get_solution(T, u0=u, v0=v, p0=p)
        torch.cuda.synchronize()
        t_solve = time.perf_counter() - t0
        stages.append({"Re": Re, "newton_iters": ns._k, "history": ns.newton_history, "solve_s": t_solve})
        print(f"stage Re={Re:g}: {ns._k} Newton iterations, {t_solve:.1f} s", flush=True)
    t_solve = time.perf_counter() - t_all
    stride = 97
    out = {"config": f"lid-driven cavity Re={args.Re:g}, {args.ne}x{args.ne} elements, P={args.P}",
           "schur_precond": args.schur_precond,
           "N": ns.N, "newton_iters": ns._k, "history": ns.newton_history, "stages": stages,
           "setup_s": t_setup, "solve_s": t_solve,
           "norm_u": float(np.linalg.norm(u)), "norm_v": float(np.linalg.norm(v)), "norm_p": float(np.linalg.norm(p)),
           "sample_stride": stride, "device": torch.cuda.get_device_name(0)}
    if args.Re == 1000.0:
        du, dv, up, vp = ghia_deviation(ns, u, v)
        out.update(ghia_max_dev_u=du, ghia_max_dev_v=dv, ghia_u=up, ghia_v=vp)
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f)
        np.savez_compressed(os.path.splitext(args.out)[0] + ".npz", u=u[::stride], v=v[::stride], p=p[::stride])


if __name__ == "__main__":
    main()
