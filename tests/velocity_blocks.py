"""Test helper (not a test module): the static-condensation pieces of a velocity Jacobian,
extracted from the oracle's assembled SciPy matrix, in sem_velocity_blocks' layout
(sem_amd/csrc/ns_velocity.hip), and the inverse map (pieces -> dense matrix)."""
import numpy as np


def _idx(N, NY, c, gx, gy):
    return c * N + gx * NY + gy


def extract(J, P, nex, ney, ncomp=2):
    """Pieces of the ncomp N x ncomp N matrix J (dense ndarray)."""
    NY, NX = ney * P + 1, nex * P + 1
    N, m = NX * NY, ncomp * NY
    cg = np.arange(m)
    comp, gy = cg // NY, cg % NY
    out = {"D": np.zeros((nex + 1, m, m)), "E": np.zeros((nex, m)), "F": np.zeros((nex, m))}
    for L in range(nex + 1):
        r = _idx(N, NY, comp, L * P, gy)
        out["D"][L] = J[np.ix_(r, r)]
        if L < nex:
            r2 = _idx(N, NY, comp, (L + 1) * P, gy)
            out["E"][L] = J[r, r2]
            out["F"][L] = J[r2, r]
    if P > 1:
        nI = (P - 1) * m
        out["AII"] = np.zeros((nex, nI, nI))
        out["aIB"] = np.zeros((nex, P - 1, 2, m))
        out["aBI"] = np.zeros((nex, 2, P - 1, m))
        for e in range(nex):
            rows = np.concatenate([_idx(N, NY, comp, e * P + l, gy) for l in range(1, P)])
            out["AII"][e] = J[np.ix_(rows, rows)]
            for li, l in enumerate(range(1, P)):
                ri = _idx(N, NY, comp, e * P + l, gy)
                for s in range(2):
                    rb = _idx(N, NY, comp, e * P + s * P, gy)
                    out["aIB"][e, li, s] = J[ri, rb]
                    out["aBI"][e, s, li] = J[rb, ri]
    return out


def assemble(pieces, P, nex, ney, ncomp=2):
    """The dense ncomp N x ncomp N matrix the pieces describe (every entry they do not name is zero)."""
    NY, NX = ney * P + 1, nex * P + 1
    N, m = NX * NY, ncomp * NY
    cg = np.arange(m)
    comp, gy = cg // NY, cg % NY
    J = np.zeros((ncomp * N, ncomp * N))
    for L in range(nex + 1):
        r = _idx(N, NY, comp, L * P, gy)
        J[np.ix_(r, r)] = pieces["D"][L]
        if L < nex:
            r2 = _idx(N, NY, comp, (L + 1) * P, gy)
            J[r, r2] = pieces["E"][L]
            J[r2, r] = pieces["F"][L]
    if P > 1:
        for e in range(nex):
            rows = np.concatenate([_idx(N, NY, comp, e * P + l, gy) for l in range(1, P)])
            J[np.ix_(rows, rows)] = pieces["AII"][e]
            for li, l in enumerate(range(1, P)):
                ri = _idx(N, NY, comp, e * P + l, gy)
                for s in range(2):
                    rb = _idx(N, NY, comp, e * P + s * P, gy)
                    J[ri, rb] = pieces["aIB"][e, li, s]
                    J[rb, ri] = pieces["aBI"][e, s, li]
    return J


def oracle_velocity_jacobian(P, nex, ney, Re, seed, Lx=1.0, Ly=1.0, smooth=0.0):
    """Dirichlet-row-replaced velocity Jacobian of the oracle NS at random (u, v)
    (NavierStokes_Solver.py:123-136,176-183) and the oracle itself.  smooth > 0: a smooth cell-like field of that
    amplitude plus 1 % noise instead (the Newton coupling then small beside the stiffness, as in a real flow)."""
    from oracle import sem_oracle as O
    ns = O.NSOracle(Lx, Ly, Re, 0.0, P, nex, ney, u_N=1.0)
    r = np.random.default_rng(seed)
    u, v = r.uniform(-1, 1, ns.N), r.uniform(-1, 1, ns.N)
    if smooth:
        x, y = (np.asarray(a) for a in ns.points)
        u = smooth * (np.sin(np.pi * x / Lx) * np.sin(2 * np.pi * y / Ly) + 0.01 * u)
        v = -smooth * (np.sin(2 * np.pi * x / Lx) * np.sin(np.pi * y / Ly) + 0.01 * v)
    ns.residuals(u, v, np.zeros(ns.N), np.zeros(ns.N))
    ns.calc_jacobians(u, v)
    ns.velocity_lu()
    return ns, u, v


def oracle_cd_jacobian(P, nex, ney, Pe, seed, Lx=1.0, Ly=1.0):
    """The oracle CD's dres operator at du = dv = 0 (Sys with Dirichlet identity rows,
    ConvectionDiffusion_Solver.py:104-121) at random (u, v), as a SciPy CSR."""
    import scipy.sparse as sp
    from oracle import sem_oracle as O
    cd = O.CDOracle(Lx, Ly, Pe, P, nex, ney, T_W=0.5, T_E=-0.5)
    r = np.random.default_rng(seed)
    u, v = r.uniform(-1, 1, cd.N), r.uniform(-1, 1, cd.N)
    cd.residuals(np.zeros(cd.N), u, v)
    A = cd.Sys.tolil()
    A[cd.mask, :] = 0
    A[cd.mask, cd.mask] = 1
    return cd, sp.csr_matrix(A), u, v
