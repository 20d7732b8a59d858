"""Full-size solver fixtures from the ORACLE (oracle/sem_oracle.py, the CPU restatement pinned
against the reference's own golden vectors by tests/test_oracle_golden.py), for configurations
whose reference run is infeasible in this container: the reference's 8-D convection tensor alone is
~35 GB at 64^2 elements.

  cd64: cfg2 mesh (64 x 64, P = 8) convection-diffusion solve of the reference example's problem
        (Examples/ConvectionDiffusion_Example.py: Pe = 40, u = y - 1/2, v = 1/2 - x, T_W/T_E = +-0.5,
        mtol = 1e-7) with SciPy LGMRES on the assembled CSR (ConvectionDiffusion_Solver.py:123-170).
        Saved: N, the solution norm, strided samples, the LGMRES matvec count.

  ns8:  lid-driven cavity (Examples/NavierStokes_Example.py) at 8 x 8 elements, P = 8, Re = 400: the
        oracle's Newton iteration with SuperLU velocity solves and the Schur-complement LGMRES
        (NavierStokes_Solver.py:162-270).  Saved: u, v, p, the Newton count and residual history.

  cfg4: BASELINE cfg4 (Boussinesq, Ra = 1e6, 48 x 48 elements, P = 8 for both solvers) at the converged
        state of the device's Ra continuation (tests/golden/cfg4_state.npz: [T, u, v, p], written by
        tools/bous_solve.py after Newton 5 of the Ra = 1e6 stage, profiles/r02/bous/b48_ra1e6_part2.log).
        Saved: the oracle's coupled residual there (ConvectionDiffusion_Solver.py:73-92 with u, v from
        the NS field; NavierStokes_Solver.py:93-121 with T from the CD field; the couplers' PG group,
        OpenMDAO/Boussinesq_SequentialCoupler.py:66-73) as block norms and strided samples, and the
        oracle's CD Newton update for a seeded right-hand side -- the exact solution of the reference's
        linearised system (_get_dresiduals at du = dv = 0, Dirichlet identity rows) by a sparse direct
        solve, which the reference's LGMRES approximates to mtol sqrt(N).  The oracle's NS update (SuperLU of
        the 296,450^2 velocity Jacobian inside an LGMRES Schur solve of ~2,000 iterations) does not finish
        in this container: the SuperLU factorisation alone ran past 10 minutes, so the GPU test pins the
        device NS update by the oracle's linearised operator instead (tests/test_gpu_cfg4.py).

Usage:  python tests/golden/make_oracle_fixtures.py cd64|ns8|cfg4   (cd64: ~6 minutes, ns8: ~40 s)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def gen_cd64():
    from oracle import sem_oracle as O
    import scipy.sparse.linalg as spla
    P, ne, Pe, mtol = 8, 64, 40.0, 1e-7
    ref = O.CDOracle(1.0, 1.0, Pe, P, ne, ne, T_W=0.5, T_E=-0.5)
    x, y = ref.points
    u, v = y - 0.5, 0.5 - x
    count = [0]
    T0 = np.zeros(ref.N)
    res = ref.residuals(T0, u, v)

    def mv(d):
        count[0] += 1
        return ref.dresiduals(d)

    t0 = time.perf_counter()
    A = spla.LinearOperator((ref.N,) * 2, matvec=mv, dtype=float)
    dT, info = spla.lgmres(A, -res, atol=mtol * np.sqrt(ref.N), rtol=0, inner_m=int(ref.N * 0.3))
    if info != 0:
        raise RuntimeError("oracle LGMRES failed")
    T = T0 + dT
    stride = 97
    np.savez_compressed(os.path.join(HERE, "cd64_checksums.npz"), N=np.array(ref.N), norm_T=np.array(np.linalg.norm(T)),
                        sample_idx=np.arange(0, ref.N, stride), sample_T=T[::stride], matvecs=np.array(count[0]),
                        final_res=np.array(np.linalg.norm(ref.residuals(T, u, v))), seconds=np.array(time.perf_counter() - t0))
    print("cd64", ref.N, count[0], np.linalg.norm(T), time.perf_counter() - t0)


def gen_ns8():
    from oracle import sem_oracle as O
    P, ne, Re = 8, 8, 400.0
    ns = O.NSOracle(1.0, 1.0, Re, 0.0, P, ne, ne, u_N=1.0)
    u, v, p, hist = ns.solution(np.zeros(ns.N), mtol=1e-7, mtol_newton=1e-5)
    np.savez_compressed(os.path.join(HERE, "ns8_re400.npz"), u=u, v=v, p=p, newton_iters=np.array(len(hist) - 1),
                        res_history=np.array([h[0] for h in hist]), schur_matvecs=np.array([h[1] for h in hist]))
    print("ns8", ns.N, len(hist) - 1, [h[0] for h in hist])


CFG4 = dict(Ne=48, P=8, Re=1e3, Ra=1e6, Pr=0.71, stride=97, seed=44)


def cfg4_rhs(N, seed=CFG4["seed"]):
    """The seeded right-hand sides of the cfg4 update checks (shared with tests/test_gpu_cfg4.py)."""
    r = np.random.default_rng(seed)
    return r.uniform(-1, 1, N), tuple(r.uniform(-1, 1, N) for _ in range(3))


def gen_cfg4():
    from oracle import sem_oracle as O
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    c = CFG4
    P, ne, Re, Ra, Pr = c["P"], c["Ne"], c["Re"], c["Ra"], c["Pr"]
    x = np.load(os.path.join(HERE, "cfg4_state.npz"))["x"]
    N = (ne * P + 1) ** 2
    T, u, v, p = x[:N], x[N:2 * N], x[2 * N:3 * N], x[3 * N:]
    t0 = time.perf_counter()
    cd = O.CDOracle(1.0, 1.0, Re * Pr, P, ne, ne, T_W=0.5, T_E=-0.5)
    ns = O.NSOracle(1.0, 1.0, Re, Ra / Pr, P, ne, ne)
    rT = cd.residuals(T, u, v)
    ru, rv, rc = ns.residuals(u, v, p, T)
    R = np.concatenate((rT, ru, rv, rc))
    s = c["stride"]
    # CD update: dres_op = Sys with the Dirichlet rows as identity rows (:104-121 at du = dv = 0)
    bT, _ = cfg4_rhs(N)
    A = cd.Sys.tolil()
    A[cd.mask, :] = 0
    A[cd.mask, cd.mask] = 1
    A = A.tocsc()
    dT = spla.spsolve(A, bT)
    res_cd = np.linalg.norm(cd.dresiduals(dT) - bT)
    np.savez_compressed(os.path.join(HERE, "cfg4_oracle.npz"), N=np.array(N), DOF=np.array(4 * N),
                        R_norm=np.array(np.linalg.norm(R)),
                        R_block_norms=np.array([np.linalg.norm(a) for a in (rT, ru, rv, rc)]),
                        R_block_amax=np.array([np.abs(a).max() for a in (rT, ru, rv, rc)]),
                        sample_idx=np.arange(0, 4 * N, s), R_sample=R[::s],
                        cd_update_norm=np.array(np.linalg.norm(dT)), cd_update_sample=dT[::s],
                        cd_update_oracle_residual=np.array(res_cd), seconds=np.array(time.perf_counter() - t0))
    print("cfg4", N, np.linalg.norm(R), [np.linalg.norm(a) for a in (rT, ru, rv, rc)], np.linalg.norm(dT), res_cd,
          time.perf_counter() - t0)


if __name__ == "__main__":
    {"cd64": gen_cd64, "ns8": gen_ns8, "cfg4": gen_cfg4}[sys.argv[1]]()
