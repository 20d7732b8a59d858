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

Usage:  python tests/golden/make_oracle_fixtures.py cd64|ns8      (cd64: ~6 minutes, ns8: ~40 s)
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


if __name__ == "__main__":
    {"cd64": gen_cd64, "ns8": gen_ns8}[sys.argv[1]]()
