"""Backward error of the condensed velocity / CD Jacobian solves against SciPy's pivoting sparse LU
(VERDICT r4 item 5): eta(x) = ||J x - b||_inf / (||J||_inf ||x||_inf + ||b||_inf), the normwise backward error,
beside the forward error against spsolve and cond_inf(J).  The forward error is at most ~cond * eta, so a
solve whose eta is at the rounding level and whose forward error is cond * eps is exact for a nearby matrix:
the distance to SuperLU is the conditioning's, not the factor's.  CPU: the torch path of
VelocityJacobianSolver with the GPU's edge choice (block LU of the edge Schur systems, no inter-block
pivoting: edge_dense_max = 0, block-Thomas factors kept)."""
import os
import sys

import numpy as np
import scipy.sparse.linalg as spla
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def eta(J, x, b):
    r = J @ x - b
    return np.abs(r).max() / (np.abs(J).sum(axis=1).max() * np.abs(x).max() + np.abs(b).max())


def one(P, nex, ney, Re, ncomp):
    from sem_amd.solvers.velocity_solve import VelocityJacobianSolver
    from velocity_blocks import extract, oracle_cd_jacobian, oracle_velocity_jacobian
    if ncomp == 2:
        ns, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex + ney)
        J = ns.Jvelo.tocsr()
    else:
        _, J, _, _ = oracle_cd_jacobian(P, nex, ney, Re, seed=P + nex)
    Jd = J.toarray()
    pcs = {k: torch.as_tensor(v) for k, v in extract(Jd, P, nex, ney, ncomp=ncomp).items()}
    ch = VelocityJacobianSolver(P, nex, ney, "cpu", ncomp=ncomp)
    cond = ch.condense_dense(pcs["AII"])

    def fill(blocks, cols):
        c0, c1 = cols
        for k in ("D", "aIB", "aBI", "E", "F"):
            blocks[k].copy_(pcs[k])
        for k, v in cond.items():
            blocks[k].copy_(v[c0:c1])
    ch.edge_dense_max, ch.edge_solve = 0, "thomas"
    ch.factor_condensed(fill)
    b = np.random.default_rng(11).uniform(-1, 1, J.shape[0])
    if ncomp == 2:
        n = J.shape[0] // 2
        x = np.hstack([t.numpy() for t in ch.solve(torch.as_tensor(b[:n]), torch.as_tensor(b[n:]))])
    else:
        x = ch.solve1(torch.as_tensor(b)).numpy()
    xs = spla.spsolve(J.tocsc(), b)
    xd = np.linalg.solve(Jd, b)
    c = np.linalg.cond(Jd, np.inf)
    fe = np.abs(x - xs).max() / np.abs(xs).max()
    print(f"P={P} {nex}x{ney} Re/Pe={Re:g} ncomp={ncomp}: cond_inf {c:.2e}  eta(ours) {eta(Jd, x, b):.2e}  "
          f"eta(SuperLU) {eta(Jd, xs, b):.2e}  eta(LAPACK) {eta(Jd, xd, b):.2e}  fwd(ours vs SuperLU) {fe:.2e}  "
          f"fwd(LAPACK vs SuperLU) {np.abs(xd - xs).max() / np.abs(xs).max():.2e}  edge_thomas {ch._edge_thomas}",
          flush=True)


if __name__ == "__main__":
    for case in [(4, 3, 1, 100.0), (6, 2, 2, 1000.0), (8, 2, 3, 500.0), (12, 2, 5, 100.0), (3, 3, 4, 50.0),
                 (7, 2, 8, 200.0)]:
        for nc in (2, 1):
            one(*case, nc)
