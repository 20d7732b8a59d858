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


def _cd_like(n, seed):
    rng = np.random.default_rng(seed)
    A = np.diag(np.linspace(1, 60, n)) + 0.04 * rng.standard_normal((n, n))
    return torch.from_numpy(A).cuda(), torch.from_numpy(rng.standard_normal(n)).cuda()


@pytest.mark.parametrize("eta", [1e-4, 2.0])
def test_pipelined_gmres_matches_unpipelined(gpu, monkeypatch, eta):
    """the pipelined step (speculative v_{k+1} and matvec queued before the host waits) against
    SEM_GMRES_PIPELINE=0 on the same preconditioned system, with the reorthogonalisation firing on every step
    (REORTH_ETA = 2: each speculation is thrown away and redone) and without.  Same iterations, x to rounding;
    the dropped speculations are reported in `discarded`, not in `matvecs`."""
    import sem_amd.krylov as K
    A, b = _cd_like(500, 9)
    d = 1.0 / torch.diagonal(A)
    monkeypatch.setattr(K, "REORTH_ETA", eta)
    out = {}
    for pipe in ("0", "1"):
        monkeypatch.setenv("SEM_GMRES_PIPELINE", pipe)
        calls = [0]

        def mv(v):
            calls[0] += 1
            return A @ v
        r = K.gmres(mv, b, atol=1e-10, restart=300, maxiter=2000, precond=lambda v: d * v)
        assert r.info == 0
        assert calls[0] == r.matvecs + r.discarded
        out[pipe] = r
    r0, r1 = out["0"], out["1"]
    assert r0.iters == r1.iters and r0.matvecs == r1.matvecs and r0.discarded == 0
    assert (r0.x - r1.x).abs().max().item() < 1e-10
    if eta > 1:
        assert r1.reorth >= r1.iters - 1 and r1.discarded >= r1.reorth - 1
    else:
        assert r1.discarded == 1          # the speculation past convergence


def test_pipelined_gmres_exact_breakdown(gpu):
    """Exact breakdown on the pipelined path: b = e_j of a power-of-two diagonal operator makes w = 4 v_0 - 4 v_0
    exactly zero after the first step; the speculative v_1 divides by one, not by zero, and is dropped; the answer
    is exact.  A 3-dimensional invariant subspace then stops after 3 steps (rounding-level ||w||)."""
    from sem_amd.krylov import gmres
    n = 300
    D = torch.diag(2.0 ** torch.arange(n, dtype=torch.float64) % 7 + 1).cuda()
    D[150, 150] = 4.0
    b = torch.zeros(n, dtype=torch.float64, device="cuda")
    b[150] = 1.0
    seen = []

    def mv(v):
        seen.append(bool(torch.isfinite(v).all()))
        return D @ v
    r = gmres(mv, b, atol=0.0, restart=40, maxiter=100)
    assert r.info == 0 and r.iters == 1 and all(seen) and r.discarded == 1
    assert torch.equal(D @ r.x, b)
    b3 = torch.zeros(n, dtype=torch.float64, device="cuda")
    b3[[3, 150, 290]] = torch.tensor([1.0, -2.0, 0.5], dtype=torch.float64, device="cuda")
    D3 = torch.diag(torch.linspace(1, 5, n, dtype=torch.float64)).cuda()
    r3 = gmres(lambda v: D3 @ v, b3, atol=1e-12, restart=40, maxiter=100)
    assert r3.iters == 3 and (D3 @ r3.x - b3).abs().max().item() < 1e-13


def test_segmented_dot2_matches_masked_products(gpu):
    """The partitioned GMRES's dot2 over owned ranges (pointer offsets, no mask) equals the masked torch
    products, for a strip (first NY entries shared) and the coupled [T | u | v | p] layout (four ranges)."""
    from sem_amd.krylov import _DeviceSweeps
    g = torch.Generator(device="cpu").manual_seed(4)
    n, k = 4 * 5003, 37
    V = (torch.rand((k + 1, n), generator=g, dtype=torch.float64) * 2 - 1).cuda()
    a, b = ((torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1).cuda() for _ in range(2))
    for segs in ([(73, n)], [(0, 5003), (5003 + 73, 2 * 5003), (2 * 5003 + 73, 3 * 5003), (3 * 5003 + 73, n)]):
        own = torch.zeros(n, dtype=torch.float64, device="cuda")
        for lo, hi in segs:
            own[lo:hi] = 1.0
        S = _DeviceSweeps(V, segs).dot2(k, a, b)
        want = torch.stack((V[:k] @ (a * own), V[:k] @ (b * own)), dim=1)
        assert (S - want).abs().max().item() <= 1e-12


@pytest.mark.parametrize("eta", [1e-4, 2.0])
def test_segmented_pipelined_gmres_matches_plain(gpu, monkeypatch, eta):
    """the partitioned Krylov path -- GMRES on owned segments through DistributedInner, its reduce on the
    device (no host staging, so the pipelined step runs) -- against plain GMRES on the same system, with and without
    the forced reorthogonalisation (REORTH_ETA = 2).  One rank and segments covering the whole vector: the
    partitioned arithmetic must give plain GMRES's iterations and x to rounding."""
    import sem_amd.krylov as K
    from sem_amd.parallel import DistributedInner
    A, b = _cd_like(600, 13)
    d = 1.0 / torch.diagonal(A)
    n = b.numel()
    monkeypatch.setattr(K, "REORTH_ETA", eta)
    inner = DistributedInner(None, (n, "cuda"), None, segments=[(0, 250), (250, 600)])
    assert inner.bdev is None            # no host staging: the pipelined step is taken
    ref = K.gmres(lambda v: A @ v, b, atol=1e-10, restart=300, maxiter=2000, precond=lambda v: d * v)
    got = K.gmres(lambda v: A @ v, b, atol=1e-10, restart=300, maxiter=2000, precond=lambda v: d * v, inner=inner)
    assert ref.info == 0 and got.info == 0
    assert abs(got.iters - ref.iters) <= 1
    assert got.discarded >= 1            # the pipeline ran (its speculation past convergence was dropped)
    assert (got.x - ref.x).abs().max().item() < 1e-9
    if eta > 1:
        assert got.reorth >= got.iters - 1
