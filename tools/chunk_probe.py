"""Diagnostic: the condensed direct solve of a CD Jacobian (ncomp = 1) and of an NS velocity Jacobian,
factored in one shot and column-chunked (VelocityJacobianSolver.factor_from budgets), on meshes where
both fit; relative residual of each solve through the fused Jacobian apply.

python tools/chunk_probe.py --ne 64 --P 12
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
    ap.add_argument("--ne", type=int, default=64)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--chunks", default="0,1,3,6")
    args = ap.parse_args()
    from sem_amd.solvers import ConvectionDiffusionSolver
    from sem_amd.solvers.velocity_solve import VelocityJacobianSolver
    cd = ConvectionDiffusionSolver(1.0, 1.0, 710.0, args.P, args.ne, args.ne, T_W=0.5, T_E=-0.5, mtol=1e-13)
    N = cd.N
    r = np.random.default_rng(3)
    cd._get_residuals(np.zeros(N), np.zeros(N), np.zeros(N))
    m = cd._mesh
    cX, cu, cY, cv, d = cd._Sys._coeffs()
    fill = lambda b, cols: m.velocity_blocks(b, cols=cols, c_mass=cd._Sys.cM, c_stiff=cd._Sys.cK, c_gradx=cX, cu=cu,  # noqa: E731
                                             c_grady=cY, cv=cv, juu=d, ncomp=1, **cd._dir.kw())
    b = cd._dev(r.uniform(-1, 1, N))
    for ch in (int(c) for c in args.chunks.split(",")):
        vs = VelocityJacobianSolver(args.P, args.ne, args.ne, m.device, ncomp=1)
        per = vs.nI * vs.nI * 8 + 3 * vs.nI * 2 * vs.m * 8
        vs.factor_from(fill, budget_bytes=(1 << 50) if ch == 0 else ch * per)
        x = vs.solve1(b)
        res = float((cd._get_dresiduals(x) - b).abs().max() / b.abs().max())
        print(json.dumps({"mesh": f"{args.ne}^2 P={args.P}", "chunk_cols": ch or "all", "rel_residual": res}),
              flush=True)
        del vs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
