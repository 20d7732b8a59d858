"""CPU probe of Schur-complement preconditioners for the NS Newton update (oracle only).

The reference preconditions the pressure Schur complement S = dres_cont(-J^-1 G dp, dp)
(NavierStokes_Solver.py:194-212) with the mass diagonal.  This probe linearises the oracle at a
converged Re=100 lid-driven flow, builds S for higher Re with SuperLU velocity solves, and counts
right-preconditioned GMRES matvecs (sem_amd.krylov.gmres, the device solver's algorithm, run on CPU
tensors) for a consistent right-hand side with several preconditioners:
  mass  the reference's M^-1 (pinned row identity)
  pcd1  M^-1 F_p A_p^-1      pcd2  A_p^-1 F_p M^-1      (pressure convection-diffusion, Elman)
  pcd3/pcd4  the same with the replaced rows (boundary K rows, the pin) routed through A_p^-1 alone
  lapl  A_p^-1 alone
A_p = K with the pinned row, F_p = Sys = K + Re (u G_x + v G_y).  pcd4 is what NavierStokesSolver
uses (schur_precond="pcd").

python tools/pcd_probe.py P N_e Re1,Re2,...
"""
import sys, time
import numpy as np, scipy.sparse as sp, scipy.sparse.linalg as spla, torch
sys.path.insert(0, '/root/repo')
from oracle import sem_oracle as O
from sem_amd.krylov import gmres

P, ne = int(sys.argv[1]), int(sys.argv[2])
Res = [float(r) for r in sys.argv[3].split(',')]
ns = O.NSOracle(1.0, 1.0, 100.0, 0.0, P, ne, ne, u_N=1.0)
N = ns.N
T = np.zeros(N)
u, v, p, hist = ns.solution(T, mtol=1e-8, mtol_newton=1e-6)
print(f"Re 100: newton {len(hist)-1}, schur matvecs {[h[1] for h in hist]}", flush=True)
for Re in Res:
    ns = O.NSOracle(1.0, 1.0, Re, 0.0, P, ne, ne, u_N=1.0)
    ns.residuals(u, v, p, T)
    ns.calc_jacobians(u, v)
    ns.velocity_lu()
    Z = np.zeros(N)
    rng = np.random.default_rng(0)
    ru, rv, rc = (rng.uniform(-1, 1, N) for _ in range(3))
    pass
    def schur(dp):
        fx, fy = ns.solve_velocity(*ns.dresiduals(Z, Z, dp)[:2])
        return ns.dresiduals(-fx, -fy, dp)[2]
    b = schur(rc)
    Md = ns.M.diagonal()
    mp, mb = ns.mask_p, ns.mask_bound
    def mass(c):
        z = c / Md; z[mp] = c[mp]; return z
    Ap = ns.K.tolil(); Ap[mp, :] = 0; Ap[mp, mp] = 1; Ap = Ap.tocsc(); Aplu = spla.splu(Ap)
    Fp = (ns.K + ns.Re * (O.conv_left(ns.Gx, u) + O.conv_left(ns.Gy, v))).tocsr()
    def pcd1(c):   # M^-1 Fp K^-1
        z = Fp @ Aplu.solve(c); z = z / Md; z[mp] = c[mp]; return z
    def pcd2(c):   # K^-1 Fp M^-1
        y = c / Md; y[mp] = 0; return Aplu.solve(Fp @ y) + np.where(mp, c, 0)
    def pcd3(c):   # interior rows PCD, boundary rows K^-1 part
        ci = c.copy(); ci[mb] = 0; ci[mp] = 0
        z = Fp @ Aplu.solve(ci); z = z / Md
        cb = np.zeros(N); cb[mb] = c[mb]; cb[mp] = c[mp]
        return z + Aplu.solve(cb)
    def pcd4(c):
        y = c / Md; y[mb] = 0; y[mp] = 0
        z = Aplu.solve(Fp @ y)
        cb = np.zeros(N); cb[mb] = c[mb]; cb[mp] = c[mp]
        return z + Aplu.solve(cb)
    def lapl(c):  # K^-1 alone
        return Aplu.solve(c)
    tb = torch.as_tensor(b)
    for name, pc in [("mass", mass), ("pcd1", pcd1), ("pcd2", pcd2), ("pcd3", pcd3), ("pcd4", pcd4), ("lapl", lapl)]:
        t0 = time.perf_counter()
        r = gmres(lambda x: torch.as_tensor(schur(x.numpy())), tb, atol=1e-10 * np.linalg.norm(b), rtol=0.0,
                  restart=1500, maxiter=1500, precond=lambda x: torch.as_tensor(pc(x.numpy())))
        res = np.linalg.norm(schur(r.x.numpy()) - b) / np.linalg.norm(b)
        print(f"Re {Re} {name}: info {r.info} matvecs {r.matvecs} rel res {res:.2e} ({time.perf_counter()-t0:.1f}s)", flush=True)
