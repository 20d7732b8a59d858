"""Boussinesq natural convection (NS + CD coupled) on the device: cfg4 is Ra = 1e6, 48 x 48
elements, P = 8 (Examples/Boussinesq_Sequential_Example.py:22-37 at BASELINE.json's configuration),
through sem_amd.solvers.boussinesq.BoussinesqCoupler (the OpenMDAO coupler's algorithm).

python tools/bous_solve.py --ne 48 --P 8 --Ra 1e6 --continuation 1e3,1e4,1e5 [--mode JNK]
Each stage starts from the previous stage's solution.  Reports Newton iterations, wall time and
u_max*Re*Pr, v_max*Re*Pr on the example's 101 x 101 plot grid (the numbers the reference example
prints, to compare with de Vahl Davis 1983: Ra = 1e6 -> 64.63 and 219.36).
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
    ap.add_argument("--ne", type=int, default=48)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--Ra", type=float, default=1e6)
    ap.add_argument("--Re", type=float, default=1e3)
    ap.add_argument("--Pr", type=float, default=0.71)
    ap.add_argument("--mode", default="JNK")
    ap.add_argument("--continuation", default="")
    ap.add_argument("--mtol-internal", type=float, default=1e-13)
    ap.add_argument("--out", default="")
    ap.add_argument("--schur-precond", default="mass", choices=["pcd", "mass"])
    ap.add_argument("--iprint", type=int, default=1)
    ap.add_argument("--x0", default="", help="start from a saved state (.npy of [T, u, v, p])")
    ap.add_argument("--ckpt", default="", help="directory for each finished stage's state (bous_<ne>_<Ra>.npy) "
                                                 "and each Newton step's (bous_<ne>_<Ra>_newton.npy)")
    ap.add_argument("--resume", type=int, default=0, help="--x0 is a mid-stage Newton state: no initial pass")
    args = ap.parse_args()
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    stages = []
    x = np.load(args.x0) if args.x0 else None
    t_all = time.perf_counter()
    for Ra in [float(r) for r in args.continuation.split(",") if r] + [args.Ra]:
        t0 = time.perf_counter()
        c = BoussinesqCoupler(1.0, 1.0, args.Re, Ra, args.Pr, args.P, args.ne, args.ne, args.P, args.ne, args.ne,
                              mode=args.mode, mtol_internal=args.mtol_internal, iprint=args.iprint,
                              schur_precond=args.schur_precond)
        if args.iprint >= 2:
            c.cd._progress = c.ns._progress = 500
            c.ns._iprint = list(c.ns._iprint) + ["LU_suc"]   # factor times and the refinement gate's backward error
        def ckpt(xs, k, Ra=Ra):
            if args.ckpt:
                os.makedirs(args.ckpt, exist_ok=True)
                np.save(os.path.join(args.ckpt, f"bous_{args.ne}_{Ra:g}_newton.npy"), xs)
                print(f"checkpoint: Ra={Ra:g} after Newton {k} ({time.perf_counter() - t0:.0f} s)", flush=True)

        T, u, v, p = c.solve(x, checkpoint=ckpt, resume=bool(args.resume) and not stages)
        x = np.concatenate((T, u, v, p))
        dt = time.perf_counter() - t0
        xp, yp = np.meshgrid(np.linspace(0, 1, 101), np.linspace(0, 1, 101), indexing="ij")
        up = np.asarray(c.ns._get_interpol(u, (xp, yp)))
        vp = np.asarray(c.ns._get_interpol(v, (xp, yp)))
        st = {"Ra": Ra, "newton_iters": c.iterations, "seconds": dt, "u_max_RePr": float(up.max() * args.Re * args.Pr),
              "v_max_RePr": float(vp.max() * args.Re * args.Pr), "timing": c.timing, "calls": c.calls}
        stages.append(st)
        print(json.dumps(st), flush=True)
        if args.ckpt:
            os.makedirs(args.ckpt, exist_ok=True)
            np.save(os.path.join(args.ckpt, f"bous_{args.ne}_{Ra:g}.npy"), x)
    out = {"config": f"Boussinesq {args.mode} Ra={args.Ra:g}, {args.ne}x{args.ne} elements, P={args.P}",
           "schur_precond": args.schur_precond,
           "N": int(c.Ncd), "DOF": int(c.DOF), "stages": stages, "seconds": time.perf_counter() - t_all,
           "norm_T": float(np.linalg.norm(T)), "norm_u": float(np.linalg.norm(u)), "norm_v": float(np.linalg.norm(v)),
           "device": torch.cuda.get_device_name(0)}
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f)
        np.savez_compressed(os.path.splitext(args.out)[0] + ".npz", T=T[::97], u=u[::97], v=v[::97])


if __name__ == "__main__":
    main()
