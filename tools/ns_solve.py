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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=32)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--Re", type=float, default=1000.0)
    ap.add_argument("--mtol", type=float, default=1e-7)
    ap.add_argument("--mtol-newton", type=float, default=1e-5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    t0 = time.perf_counter()
    ns = NavierStokesSolver(1.0, 1.0, args.Re, 0.0, args.P, args.ne, args.ne, u_N=1.0, mtol=args.mtol,
                            mtol_newton=args.mtol_newton, iprint=["NEWTON_iter", "NEWTON_suc", "LU_suc"])
    t_setup = time.perf_counter() - t0
    T = np.zeros(ns.N)
    t0 = time.perf_counter()
    u, v, p = ns._get_solution(T)
    torch.cuda.synchronize()
    t_solve = time.perf_counter() - t0
    stride = 97
    out = {"config": f"lid-driven cavity Re={args.Re:g}, {args.ne}x{args.ne} elements, P={args.P}",
           "N": ns.N, "newton_iters": ns._k, "history": ns.newton_history,
           "setup_s": t_setup, "solve_s": t_solve,
           "norm_u": float(np.linalg.norm(u)), "norm_v": float(np.linalg.norm(v)), "norm_p": float(np.linalg.norm(p)),
           "sample_stride": stride, "device": torch.cuda.get_device_name(0)}
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f)
        np.savez_compressed(os.path.splitext(args.out)[0] + ".npz", u=u[::stride], v=v[::stride], p=p[::stride])


if __name__ == "__main__":
    main()
