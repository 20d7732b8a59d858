"""Device GMRES (sem_amd/krylov.py) on CPU tensors against SciPy, on the reference's own
CD and NS-like systems built by the oracle (the algorithm is device-agnostic)."""
import math
import numpy as np
import pytest
import scipy.sparse.linalg as spla
import torch

from oracle import sem_oracle as O
from sem_amd.krylov import gmres


def _cd_system(P=4, ne=4, Pe=40.0):
    cd = O.CDOracle(1.0, 1.0, Pe, P, ne, ne, T_W=0.5, T_E=-0.5)
    x, y = cd.points
    T = np.zeros(cd.N)
    res = cd.residuals(T, y - 0.5, 0.5 - x)
    A = spla.LinearOperator((cd.N,) * 2, matvec=lambda d: cd.dresiduals(d), dtype=float)
    return cd, A, -res


def test_gmres_solves_cd_update_like_reference():
    cd, A, b = _cd_system()
    atol = 1e-7 * np.sqrt(cd.N)
    mv = lambda v: torch.from_numpy(A.matvec(v.numpy()))  # noqa: E731
    r = gmres(mv, torch.from_numpy(b), atol=atol, restart=int(0.3 * cd.N))
    assert r.info == 0
    true_res = np.linalg.norm(A.matvec(r.x.numpy()) - b)
    assert true_res <= atol * 1.0001
    ref, info = spla.lgmres(A, b, atol=atol, rtol=0, inner_m=int(0.3 * cd.N))
    assert info == 0
    assert np.abs(r.x.numpy() - ref).max() < 1e-5


def test_gmres_restarts_and_preconditioner():
    rng = np.random.default_rng(0)
    n = 200
    M = np.diag(np.linspace(1, 100, n)) + 0.05 * rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    d = torch.from_numpy(1.0 / np.diag(M).copy())
    mv = lambda v: torch.from_numpy(M @ v.numpy())  # noqa: E731
    r = gmres(mv, torch.from_numpy(b), atol=1e-10, restart=15, precond=lambda v: d * v, maxiter=5000)
    assert r.info == 0 and np.linalg.norm(M @ r.x.numpy() - b) <= 1e-10 * 1.0001
    r2 = gmres(mv, torch.from_numpy(b), atol=1e-300, restart=5, maxiter=7)
    assert r2.info == 7  # not converged: iterations performed, as SciPy reports


def test_gmres_left_matches_scipy_left_preconditioned():
    """krylov.gmres_left restates SciPy's gmres (left preconditioner M): same stopping rule,
    converged to the same solution, M only ever applied to vectors in range(A)."""
    from sem_amd.krylov import gmres_left
    rng = np.random.default_rng(3)
    n = 300
    A = np.diag(np.linspace(1, 200, n)) + 0.1 * rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    dinv = 1.0 / np.diag(A)
    mv = lambda v: torch.from_numpy(A @ v.numpy())  # noqa: E731
    r = gmres_left(mv, torch.from_numpy(b), atol=1e-9, restart=20, maxiter=500,
                   precond=lambda v: torch.from_numpy(dinv * v.numpy()))
    assert r.info == 0 and np.linalg.norm(A @ r.x.numpy() - b) <= 1e-9
    M = spla.LinearOperator((n, n), matvec=lambda v: dinv * v, dtype=float)
    ref, info = spla.gmres(A, b, atol=1e-9, rtol=0, restart=20, maxiter=500, M=M)
    assert info == 0
    assert np.abs(r.x.numpy() - ref).max() < 1e-8
    # not converged: info = maxiter (restarts), as SciPy reports
    r2 = gmres_left(mv, torch.from_numpy(b), atol=1e-300, restart=4, maxiter=3)
    assert r2.info == 3
    assert gmres_left(mv, torch.zeros(n, dtype=torch.float64)).info == 0


def test_gmres_left_cd_system():
    from sem_amd.krylov import gmres_left
    cd, A, b = _cd_system()
    atol = 1e-9 * np.sqrt(cd.N)
    mv = lambda v: torch.from_numpy(A.matvec(v.numpy()))  # noqa: E731
    r = gmres_left(mv, torch.from_numpy(b), atol=atol, restart=20, maxiter=5000)
    assert r.info == 0 and np.linalg.norm(A.matvec(r.x.numpy()) - b) <= atol


def test_gmres_basis_stays_orthonormal_on_ill_conditioned_system():
    """the Gram-matrix second pass of CGS2 cannot see the rounding error of the first
    subtraction.  On a badly conditioned, non-normal system (Krylov vectors nearly dependent, the
    first pass cancelling strongly) the basis must stay orthonormal and the true residual must meet
    the tolerance."""
    import torch
    from sem_amd.krylov import gmres
    n = 400
    g = torch.Generator().manual_seed(0)
    Q, _ = torch.linalg.qr(torch.randn(n, n, dtype=torch.float64, generator=g))
    ev = torch.logspace(-8, 0, n, dtype=torch.float64)              # cond 1e8
    A = Q @ torch.diag(ev) @ Q.T + 1e-3 * torch.triu(torch.randn(n, n, dtype=torch.float64, generator=g), 1)
    b = torch.randn(n, dtype=torch.float64, generator=g)
    basis = []
    r = gmres(lambda v: A @ v, b, atol=1e-10 * torch.linalg.vector_norm(b).item(), restart=n, basis_out=basis)
    assert r.info == 0
    assert torch.linalg.vector_norm(A @ r.x - b).item() <= 1.0001e-10 * torch.linalg.vector_norm(b).item()
    for V in basis:
        E = V @ V.T - torch.eye(V.shape[0], dtype=torch.float64)
        assert E.abs().max().item() < 1e-10, E.abs().max().item()


@pytest.mark.parametrize("precond", [False, True])
def test_gcro_recycling_sequence(precond):
    """sem_amd.krylov.gcro with a Recycle: every solve of a sequence with one operator meets the
    tolerance, the recycle space keeps A U = C and C^T C = I, and later solves of related right-hand
    sides take no more iterations than the first."""
    import torch
    from sem_amd.krylov import Recycle, gcro
    n = 500
    g = torch.Generator().manual_seed(3)
    A = (torch.eye(n, dtype=torch.float64) * 2 + 0.3 * torch.randn(n, n, dtype=torch.float64, generator=g) / n ** 0.5
         + torch.diag(torch.linspace(0, 5, n, dtype=torch.float64)))
    M = 1.0 / torch.linspace(1, 3, n, dtype=torch.float64)
    pc = (lambda v: M * v) if precond else None
    rc = Recycle(n, torch.float64, "cpu", 400)
    b = torch.randn(n, dtype=torch.float64, generator=g)
    its = []
    for _ in range(6):
        r = gcro(lambda v: A @ v, b, atol=1e-10, restart=30, precond=pc, recycle=rc)
        assert r.info == 0 and torch.linalg.vector_norm(A @ r.x - b).item() <= 1.0001e-10
        its.append(r.iters)
        b = b + 0.2 * torch.randn(n, dtype=torch.float64, generator=g)
    rc.absorb()
    C, U = rc.buf[:rc.k], rc.U[:rc.k]
    assert (C @ C.T - torch.eye(rc.k, dtype=torch.float64)).abs().max().item() < 1e-12
    AU = (A @ (U.T)).T
    assert (AU - C).abs().max().item() < 1e-12
    assert max(its[1:]) <= its[0]


def test_partitioned_krylov_sizes_ignore_the_local_length():
    """A partitioned solve (inner given) must size nothing from its local length: ranks holding strips of
    different sizes would leave the Arnoldi loop at different iterations and their collectives would
    mismatch (the world-8 gloo NS test with one-column strips).  The restart is taken as given (not clamped to
    the local N) and maxiter is required."""
    from sem_amd.krylov import _sizes, gmres_left
    assert _sizes(10, 40, None, None, 100) == (10, 100)          # one process: clamped to N, default cap 10 N
    assert _sizes(10, 40, 500, lambda A, w: A @ w, 100) == (40, 500)
    with pytest.raises(ValueError, match="maxiter"):
        _sizes(10, 40, None, lambda A, w: A @ w, 100)
    A = torch.eye(5, dtype=torch.float64) * 2.0
    b = torch.ones(5, dtype=torch.float64)
    with pytest.raises(ValueError, match="maxiter"):
        gmres(lambda v: A @ v, b, atol=1e-12, inner=lambda V, w: V @ w)
    with pytest.raises(ValueError, match="maxiter"):
        gmres_left(lambda v: A @ v, b, atol=1e-12, inner=lambda V, w: V @ w)
    # a restart above the local length still converges on the local system (the Krylov space saturates)
    r = gmres(lambda v: A @ v, b, atol=1e-12, restart=40, maxiter=100, inner=lambda V, w: V @ w)
    assert r.info == 0 and torch.allclose(r.x, b / 2.0)


def test_strip_solver_never_captures_over_host_collectives():
    """Under gloo the strip solve's all-gather goes through the host, so StripLineSolver.capture declines
    (a capture there failed part-way after a collective warm-up)."""
    from sem_amd.solvers.strip_solve import StripLineSolver
    vs = StripLineSolver(4, 4, 2, "cpu", [0, 2, 4], 0, dist=None, gather_device="cpu")
    vs.factored = True
    assert vs.capture() is False


def test_givens_column_c_matches_python_loop():
    """sem_givens_column (the library's host code) applies the same rotations in the same order as the Python loop
    it replaced: equal results on a sequence of columns, to the last bit except through hypot (one rounding)."""
    import sem_amd.krylov as K
    rng = np.random.default_rng(3)
    n = 60
    cs_c, sn_c, g_c = np.zeros(n), np.zeros(n), np.zeros(n + 1)
    cs_p, sn_p, g_p = np.zeros(n), np.zeros(n), np.zeros(n + 1)
    g_c[0] = g_p[0] = 1.7
    K.givens_column(np.ones(2), np.zeros(1), np.zeros(1), np.zeros(2), 0)   # loads the library once
    saved = list(K._GIVENS)
    for k in range(n):
        col = rng.standard_normal(k + 2)
        c1, c2 = col.copy(), col.copy()
        K.givens_column(c1, cs_c, sn_c, g_c, k)
        K._GIVENS[:] = [None]          # the interpreter fallback
        K.givens_column(c2, cs_p, sn_p, g_p, k)
        K._GIVENS[:] = saved
        assert np.allclose(c1, c2, rtol=1e-14, atol=1e-15)
    assert saved and saved[0] is not None   # the C path was the one under test
    assert np.allclose(g_c, g_p, rtol=1e-13, atol=1e-300) and np.allclose(cs_c, cs_p, rtol=1e-14)


def test_flexible_path_with_a_varying_preconditioner():
    """linear_precond=False keeps Z = M_k^-1 V (flexible GMRES), the only correct form when the
    preconditioner changes between applications (an inner iterative solve).  With a preconditioner that varies
    per call the flexible path meets the tolerance on the TRUE residual; the linear form (correction
    M^-1 (V y)) is not meant for it.  With a fixed preconditioner both forms give SciPy's solution."""
    rng = np.random.default_rng(11)
    n = 160
    A = np.diag(np.linspace(1, 80, n)) + 0.05 * rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    At, bt = torch.from_numpy(A), torch.from_numpy(b)
    d = torch.from_numpy(1.0 / np.diag(A).copy())
    calls = [0]

    def varying(v):                      # a different diagonal scaling on every call
        calls[0] += 1
        return d * v * (1.0 + 0.3 * np.sin(calls[0]))

    r = gmres(lambda v: At @ v, bt, atol=1e-10, restart=60, maxiter=2000, precond=varying, linear_precond=False)
    assert r.info == 0
    assert np.linalg.norm(A @ r.x.numpy() - b) <= 1e-10 * 1.0001
    ref, info = spla.gmres(A, b, atol=1e-11, rtol=0, restart=60, maxiter=200)
    assert info == 0
    for lin in (True, False):
        rf = gmres(lambda v: At @ v, bt, atol=1e-10, restart=60, maxiter=2000, precond=lambda v: d * v,
                   linear_precond=lin)
        assert rf.info == 0 and np.abs(rf.x.numpy() - ref).max() < 1e-8


def test_gmres_forced_reorthogonalisation_and_breakdown(monkeypatch):
    """The reorthogonalisation branch on every step (REORTH_ETA > 1) gives the same solution as the default, and
    an exact breakdown (b in a 3-dimensional invariant subspace) stops after 3 iterations with the exact answer."""
    import sem_amd.krylov as K
    rng = np.random.default_rng(2)
    n = 120
    A = torch.from_numpy(np.diag(np.linspace(1, 30, n)) + 0.02 * rng.standard_normal((n, n)))
    b = torch.from_numpy(rng.standard_normal(n))
    r0 = K.gmres(lambda v: A @ v, b, atol=1e-11, restart=80, maxiter=1000)
    monkeypatch.setattr(K, "REORTH_ETA", 2.0)
    r1 = K.gmres(lambda v: A @ v, b, atol=1e-11, restart=80, maxiter=1000)
    assert r0.info == 0 and r1.info == 0 and r1.reorth >= r1.iters - 1 and r0.reorth == 0
    assert abs(r0.iters - r1.iters) <= 1 and (r0.x - r1.x).abs().max().item() < 1e-9
    monkeypatch.setattr(K, "REORTH_ETA", 1e-4)
    D = torch.diag(torch.linspace(1, 5, n, dtype=torch.float64))
    bb = torch.zeros(n, dtype=torch.float64)
    bb[[3, 50, 90]] = torch.tensor([1.0, -2.0, 0.5], dtype=torch.float64)
    rb = K.gmres(lambda v: D @ v, bb, atol=1e-12, restart=40, maxiter=100)
    assert rb.iters == 3 and (D @ rb.x - bb).abs().max().item() < 1e-13


class _NoisyPrecond:
    """An inexact preconditioner, as the coupler's iterative block solves are: M^-1 v = D^-1 v plus a perturbation
    of relative size `level` that differs at every application (fixed seed, so the test is deterministic)."""

    def __init__(self, d, level, seed=3):
        self.d, self.level = d, level
        self.g = torch.Generator().manual_seed(seed)
        self.calls = 0

    def __call__(self, v):
        self.calls += 1
        z = v / self.d
        if self.level:
            e = torch.rand(v.shape, generator=self.g, dtype=v.dtype) * 2 - 1
            z = z + self.level * torch.linalg.vector_norm(z) / math.sqrt(v.numel()) * e
        return z


def _jump_system(n=300, seed=5):
    r = np.random.default_rng(seed)
    A = np.diag(np.linspace(1.0, 50.0, n)) + 0.3 * r.standard_normal((n, n)) / np.sqrt(n)
    return torch.as_tensor(A), torch.as_tensor(r.standard_normal(n)), torch.as_tensor(np.diag(A).copy())


def test_gmres_left_restart_jump_safeguard():
    """gmres_left detects a jump of the preconditioned residual at a restart (the inexact-
    preconditioner failure of cfg5's coupled solve) and lets the caller tighten its preconditioner; with a consistent
    preconditioner the hook never fires and the history is bitwise the unguarded one."""
    from sem_amd.krylov import gmres_left
    A, b, d = _jump_system()
    atol = 1e-10 * float(torch.linalg.vector_norm(b))
    # consistent preconditioner: no detection, identical iterates with and without the hook
    fired = []
    r0 = gmres_left(lambda v: A @ v, b, atol=atol, restart=10, maxiter=200, precond=_NoisyPrecond(d, 0.0))
    r1 = gmres_left(lambda v: A @ v, b, atol=atol, restart=10, maxiter=200, precond=_NoisyPrecond(d, 0.0),
                    jump=lambda ratio: fired.append(ratio) or True)
    assert r0.info == 0 and r1.info == 0 and not fired and r1.jumps == 0
    assert r0.iters == r1.iters and torch.equal(r0.x, r1.x)
    # inconsistent preconditioner: the unguarded solve restarts again and again at its noise floor (5 jumps); the
    # guarded one detects the first jump, tightens the preconditioner and converges in half the iterations
    pc = _NoisyPrecond(d, 1e-2)
    bad = gmres_left(lambda v: A @ v, b, atol=atol, restart=10, maxiter=60, precond=pc, jump=lambda ratio: False)
    assert bad.jumps >= 3

    def tighten(ratio):
        pg.level *= 1e-3
        return True
    pg = _NoisyPrecond(d, 1e-2)
    good = gmres_left(lambda v: A @ v, b, atol=atol, restart=10, maxiter=60, precond=pg, jump=tighten)
    assert good.info == 0 and good.jumps >= 1 and pg.level < 1e-2
    assert torch.linalg.vector_norm(A @ good.x - b).item() <= atol
    assert good.iters < 0.7 * bad.iters         # measured: 27 against 57 iterations
