"""Krylov-basis sweep kernels (include/sem_ops.h: sem_basis_dot2, sem_basis_update) against
torch fp64 on the same operands, and the device GMRES that uses them."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,n", [(1, 1), (1, 1000), (7, 100003), (300, 4097), (65, 263169)])
def test_basis_sweeps_vs_torch(gpu, k, n):
    from sem_amd.krylov import _DeviceSweeps
    g = torch.Generator(device="cpu").manual_seed(k * 31 + n)
    V = (torch.rand((k + 3, n), generator=g, dtype=torch.float64) * 2 - 1).cuda()
    a, b, c = ((torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1).cuda() for _ in range(3))
    coef = (torch.rand(k, generator=g, dtype=torch.float64) * 2 - 1).cuda()
    sw = _DeviceSweeps(V)
    S = sw.dot2(k, a, b).clone()
    want = torch.stack((V[:k] @ a, V[:k] @ b), dim=1)
    tol = 1e-13 * max(1.0, float((V[:k].abs() @ a.abs()).max()))
    assert float((S - want).abs().max()) <= tol
    assert torch.equal(sw.dot2(k, a, b), S)  # fixed summation order: bitwise reproducible
    w = c.clone()
    sw.update(k, coef, w)
    ref = c - V[:k].T @ coef
    assert float((w - ref).abs().max()) <= 1e-13 * max(1.0, float((V[:k].abs().T @ coef.abs()).max()))


def test_device_gmres_matches_host_gmres(gpu):
    """The same right-preconditioned GMRES on CPU tensors (torch BLAS) and on the GPU (HIP sweeps)."""
    from sem_amd.krylov import gmres
    rng = np.random.default_rng(5)
    n = 400
    A = np.diag(np.linspace(1, 50, n)) + 0.05 * rng.standard_normal((n, n))
    b = rng.standard_normal(n)
    At, bt = torch.from_numpy(A), torch.from_numpy(b)
    rc = gmres(lambda v: At @ v, bt, atol=1e-10, restart=200)
    Ag, bg = At.cuda(), bt.cuda()
    rg = gmres(lambda v: Ag @ v, bg, atol=1e-10, restart=200)
    assert rc.info == 0 and rg.info == 0
    assert abs(rc.iters - rg.iters) <= 1
    assert np.abs(rg.x.cpu().numpy() - np.linalg.solve(A, b)).max() < 1e-8
