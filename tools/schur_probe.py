"""CPU probe of Schur-complement preconditioners for the NS Newton update (oracle only).

The reference preconditions the pressure Schur complement
    S dp = dres_cont(-J^-1 [G_x dp; G_y dp]_D, dp)        (NavierStokes_Solver.py:194-212)
with the mass diagonal.  Rows of S: interior continuity rows -B J^-1 G dp (B = [G_x G_y] on the velocity,
G = [G_x; G_y] on the pressure, J the velocity Jacobian with Dirichlet rows), the boundary rows K[mask,:] dp
(the artificial Neumann rows, :119,157) and the pinned row.  This probe linearises the oracle at a lid-driven
flow, builds S with SuperLU velocity solves, and counts right-preconditioned GMRES matvecs (sem_amd.krylov.gmres,
the device solver's algorithm, on CPU tensors) for a consistent right-hand side:
  mass   the reference's M^-1 (pinned row identity)
  pcd4   PCD with the replaced rows through A_p^-1 (NavierStokesSolver schur_precond="pcd")
  lsc    least-squares commutator with A_p = K (pinned) for B M^-1 G ~ -K:
         interior rows  z = -A_p^-1 B M^-1 J M^-1 G A_p^-1 c   (Elman et al.'s BFBt form, M-scaled);
         replaced rows  A_p^-1 c
  lscd   the same with diag(J)-scaled commutator: -A_p^-1 B D^-1 J D^-1 G A_p^-1 (D = velocity mass * |diag J|)
  simple SIMPLE-type: z = -(A_p^-1 scaled by the mean diagonal of J / M) on interior rows
A_p = K with the pinned row as identity.  Reports matvecs and the preconditioner's cost in solve units.

python tools/schur_probe.py P N_e Re1,Re2,...   [SEM_PROBE_TOL=1e-10]
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import sem_oracle as O  # noqa: E402
from sem_amd.krylov import gmres  # noqa: E402


def main():
    P, ne = int(sys.argv[1]), int(sys.argv[2])
    Res = [float(r) for r in sys.argv[3].split(',')]
    tol = float(os.environ.get("SEM_PROBE_TOL", "1e-10"))
    ns = O.NSOracle(1.0, 1.0, 100.0, 0.0, P, ne, ne, u_N=1.0)
    N = ns.N
    T = np.zeros(N)
    u, v, p, hist = ns.solution(T, mtol=1e-8, mtol_newton=1e-6)
    print(f"P={P} {ne}x{ne} N={N}; Re 100 state: newton {len(hist) - 1}", flush=True)
    for Re in Res:
        ns = O.NSOracle(1.0, 1.0, Re, 0.0, P, ne, ne, u_N=1.0)
        ns.residuals(u, v, p, T)
        ns.calc_jacobians(u, v)
        ns.velocity_lu()
        Z = np.zeros(N)
        rc = np.random.default_rng(0).uniform(-1, 1, N)

        def schur(dp):
            fx, fy = ns.solve_velocity(*ns.dresiduals(Z, Z, dp)[:2])
            return ns.dresiduals(-fx, -fy, dp)[2]

        b = schur(rc)
        Md = ns.M.diagonal()
        mp, mb = ns.mask_p, ns.mask_bound
        repl = mp | mb
        Ap = ns.K.tolil()
        Ap[mp, :] = 0
        Ap[mp, mp] = 1
        Aplu = spla.splu(Ap.tocsc())
        Fp = (ns.K + ns.Re * (O.conv_left(ns.Gx, u) + O.conv_left(ns.Gy, v))).tocsr()
        Gx, Gy = ns.Gx.tocsr(), ns.Gy.tocsr()
        # diagonal of the velocity Jacobian (u and v blocks) through its action on unit vectors is costly; take
        # it from the oracle's assembled blocks where present, else from F_p (the same convection-diffusion part)
        dJ = np.abs(Fp.diagonal()) + 1e-300

        def Japply(wu, wv):
            return ns.dresiduals(wu, wv, Z)[:2]

        def mass(c):
            z = c / Md
            z[mp] = c[mp]
            return z

        def pcd4(c):
            y = c / Md
            y[mb] = 0
            y[mp] = 0
            z = Aplu.solve(Fp @ y)
            cb = np.zeros(N)
            cb[mb] = c[mb]
            cb[mp] = c[mp]
            return z + Aplu.solve(cb)

        def lsc_with(scale):
            def f(c):
                ci = np.where(repl, 0.0, c)
                y = Aplu.solve(ci)
                wu, wv = (Gx @ y) / scale, (Gy @ y) / scale
                ju, jv = Japply(wu, wv)
                q = Gx @ (ju / scale) + Gy @ (jv / scale)
                q[repl] = 0.0
                z = -Aplu.solve(q)
                cb = np.where(repl, c, 0.0)
                return z + Aplu.solve(cb)
            return f

        def simple(c):
            ci = np.where(repl, 0.0, c)
            s = np.mean(dJ / Md)
            z = -s * Aplu.solve(ci)
            return z + Aplu.solve(np.where(repl, c, 0.0))

        tb = torch.as_tensor(b)
        for name, pc in [("mass", mass), ("pcd4", pcd4), ("lsc", lsc_with(Md)), ("lscd", lsc_with(Md * 0 + dJ)),
                         ("simple", simple)]:
            t0 = time.perf_counter()
            r = gmres(lambda x: torch.as_tensor(schur(x.numpy())), tb, atol=tol * np.linalg.norm(b), rtol=0.0,
                      restart=2000, maxiter=2000, precond=lambda x: torch.as_tensor(pc(x.numpy())))
            res = np.linalg.norm(schur(r.x.numpy()) - b) / np.linalg.norm(b)
            err = np.abs(r.x.numpy() - rc)[~mp].max() / np.abs(rc).max()
            print(f"Re {Re:6g} {name:6s}: info {r.info} matvecs {r.matvecs:5d} rel res {res:.2e} "
                  f"x err {err:.1e} ({time.perf_counter() - t0:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
