"""Device GMRES (sem_amd/krylov.py) on CPU tensors against SciPy, on the reference's own
CD and NS-like systems built by the oracle (the algorithm is device-agnostic)."""
import numpy as np
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
