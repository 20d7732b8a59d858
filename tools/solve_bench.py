"""End-to-end convection-diffusion solve: device operators + device GMRES against the oracle.

The reference example's problem (Examples/ConvectionDiffusion_Example.py): Pe = 40, circular flow
u = y - 1/2, v = 1/2 - x, T_W = 0.5, T_E = -0.5, on N_e x N_e elements of order P.  The reference
solves it with one Newton step: the residual Sys T (ConvectionDiffusion_Solver.py:73-92), then
SciPy LGMRES with inner_m = int(0.3 N) (:123-156, :158-170).  SURVEY.md 8(a) a13 measured 15.3 s
for that at 32^2, P=8 on one host core, 12.2 s of it in Arnoldi.

This times three paths on the same problem:
* device: ConvectionDiffusionSolver(krylov="device"), the default.  Right-preconditioned GMRES
  with its basis in HBM, every matvec the fused band apply; the preconditioner is the condensed
  direct solve of the Jacobian (precond="condensed", factor time included).
* device_gmres: the same without preconditioner (precond=None): plain GMRES.
* scipy: the same solver with krylov="scipy".  The reference's LGMRES on the host around device
  matvecs.
* oracle: CDOracle.solution on the host, the reference's own arithmetic (CSR SpMV + LGMRES).
It reports wall time and matvec count for each, and each solution's relative max difference
from the oracle's (both Krylov paths stop at the reference's atol = 1e-7 sqrt(N)).

Run:  python tools/solve_bench.py [--ne 32] [--P 8] [--oracle 1]
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
    ap.add_argument("--ne", type=int, default=32)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--Pe", type=float, default=40.0)
    ap.add_argument("--oracle", type=int, default=1, help="also time the host oracle (about 15 s at 32^2, P=8)")
    ap.add_argument("--scipy", type=int, default=1, help="also time the device-matvec + host LGMRES path")
    ap.add_argument("--plain", type=int, default=1, help="also time the unpreconditioned device GMRES")
    args = ap.parse_args()
    from oracle import sem_oracle as O
    from sem_amd.solvers import ConvectionDiffusionSolver

    P, ne, Pe = args.P, args.ne, args.Pe
    out = {"problem": f"CD example (Pe={Pe:g}, circular flow, T_W=0.5, T_E=-0.5), {ne}x{ne} elements, P={P}"}
    u_f = lambda x, y: y - 0.5  # noqa: E731
    v_f = lambda x, y: 0.5 - x  # noqa: E731
    res = {}
    paths = [("device", "device", "condensed")] + ([("device_gmres", "device", None)] if args.plain else []) \
        + ([("scipy", "scipy", None)] if args.scipy else [])
    for name, kry, pc in paths:
        cd = ConvectionDiffusionSolver(1.0, 1.0, Pe, P, ne, ne, T_E=-0.5, T_W=0.5, krylov=kry, precond=pc)
        u, v = cd._get_vector(u_f), cd._get_vector(v_f)
        cd._get_solution(u, v)  # warm-up (kernel load, caches)
        torch.cuda.synchronize()
        count = [0]
        inner = cd._get_dresiduals

        def counted(*a, **k):
            count[0] += 1
            return inner(*a, **k)

        cd._get_dresiduals = counted
        t0 = time.perf_counter()
        T = cd._get_solution(u, v)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        T = T.cpu().numpy() if isinstance(T, torch.Tensor) else np.asarray(T)
        res[name] = T
        out[name] = {"wall_s": wall, "matvecs": count[0], "N": cd.N,
                     "residual_2norm": float(np.linalg.norm(cd._get_residuals(T, u, v)))}
    if args.oracle:
        ref = O.CDOracle(1.0, 1.0, Pe, P, ne, ne, T_W=0.5, T_E=-0.5)
        u, v = ref.points[1] - 0.5, 0.5 - ref.points[0]
        t0 = time.perf_counter()
        Tref = ref.solution(u, v)
        out["oracle"] = {"wall_s": time.perf_counter() - t0, "cores": 1,
                         "kind": "port (SciPy CSR + LGMRES, the reference's arithmetic)"}
        for k, T in res.items():
            out[k]["rel_maxdiff_vs_oracle"] = float(np.abs(T - Tref).max() / np.abs(Tref).max())
        out["speedup_device_vs_oracle"] = out["oracle"]["wall_s"] / out["device"]["wall_s"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
