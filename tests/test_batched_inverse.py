"""CPU tests of the checked batched inverse of the velocity condensation
(sem_amd/solvers/velocity_solve.py: batched_inverse / _bad_blocks): a wrong block returned by the
batched library call is detected and repaired, an ill-conditioned but correct block is accepted, and a
block no route can invert accurately raises."""
import numpy as np
import pytest
import torch

from sem_amd.solvers import velocity_solve as VS


def _blocks(nb, n, seed):
    r = np.random.default_rng(seed)
    A = r.uniform(-1, 1, (nb, n, n)) + n * np.eye(n)   # well conditioned
    return torch.as_tensor(A)


def _ill(n, cond, seed):
    r = np.random.default_rng(seed)
    U, _ = np.linalg.qr(r.standard_normal((n, n)))
    V, _ = np.linalg.qr(r.standard_normal((n, n)))
    return torch.as_tensor(U @ np.diag(np.logspace(0, -np.log10(cond), n)) @ V.T)


def test_accepts_correct_and_ill_conditioned_blocks():
    A = _blocks(300, 24, 1)
    A[137] = _ill(24, 1e10, 2)
    X = VS.batched_inverse(A, max_batch=128)
    assert VS._bad_blocks(A, X).numel() == 0
    want = torch.linalg.inv(A)
    assert (X[:137] - want[:137]).abs().max() <= 1e-13 * want[:137].abs().max()
    # the ill-conditioned block: a backward-stable inverse, not necessarily the same rounding
    E = A[137] @ X[137] - torch.eye(24, dtype=torch.float64)
    assert E.abs().max() <= 8 * 24 * 24 * 2.3e-16 * A[137].abs().max() * X[137].abs().max()


def test_rejects_a_wrong_inverse():
    A = _blocks(4, 16, 3)
    X = torch.linalg.inv(A)
    X[2, 3, 5] += 1e-6 * X[2].abs().max()   # one wrong entry: residual far above n^2 eps |A||X|
    assert VS._bad_blocks(A, X).tolist() == [2]
    # the same perturbation of an ill-conditioned block is still rejected: the bound is relative
    B = _ill(16, 1e10, 4)[None]
    Y = torch.linalg.inv(B)
    Y[0, 1, 1] += 1e-3 * Y.abs().max()
    assert VS._bad_blocks(B, Y).tolist() == [0]


def test_repairs_blocks_the_batched_call_got_wrong(monkeypatch):
    """The failure seen on MI355X (tools/inv_repro.py): the batched call returns some wrong blocks
    without an error.  Simulated by corrupting, in every slice, a sampled block (which triggers the
    full check of the slice) and another one (found by that full check)."""
    A = _blocks(300, 20, 5)
    calls = []

    def corrupt(a):
        x = torch.linalg.inv(a)
        calls.append(a.shape[0])
        x[0] *= 3.0
        x[len(calls) % a.shape[0] + 1] *= 3.0
        return x, torch.zeros(a.shape[0], dtype=torch.int32)

    monkeypatch.setattr(VS, "_inverse", corrupt)
    X = VS.batched_inverse(A, max_batch=128)
    assert calls == [128, 128, 44]
    want = torch.linalg.inv(A)
    assert (X - want).abs().max() <= 1e-13 * want.abs().max()


def test_unsampled_bad_block_found_by_lu_status(monkeypatch):
    """A block the 8-block sample misses is still repaired when the LU reports it singular (info != 0) or its
    computed inverse is not finite: either sends the slice to the full check."""
    A = _blocks(300, 12, 9)
    for how in ("info", "nan"):
        def route(a):
            x = torch.linalg.inv(a)
            info = torch.zeros(a.shape[0], dtype=torch.int32)
            x[37] *= 3.0                   # never among the 8 sampled blocks of a 128-block slice
            if how == "info":
                info[37] = 5
            else:
                x[38, 0, 0] = float("nan")
            return x, info
        monkeypatch.setattr(VS, "_inverse", route)
        X = VS.batched_inverse(A, max_batch=128)
        want = torch.linalg.inv(A)
        assert (X - want).abs().max() <= 1e-13 * want.abs().max(), how


def test_raises_when_no_route_inverts(monkeypatch):
    A = _blocks(10, 8, 6)
    monkeypatch.setattr(VS, "_inverse", lambda a: (torch.zeros_like(a), None))
    real_inv = torch.linalg.inv
    monkeypatch.setattr(torch.linalg, "inv", lambda a: real_inv(a) * 2.0)
    monkeypatch.setattr(torch.linalg, "solve", lambda a, b: torch.zeros_like(b))
    with pytest.raises(RuntimeError, match="could not be inverted"):
        VS.batched_inverse(A, max_batch=4)


def test_block_inverse_matches_lu():
    """The GEMM-recursive inverse of the sweep pivots (sem_amd/linalg.py) against the pivoted LU."""
    from sem_amd.linalg import block_inverse
    r = np.random.default_rng(11)
    n = 700                                  # splits 384 | 316, then leaves of <= 256 rows
    A = torch.as_tensor(r.uniform(-1, 1, (n, n)) + 4 * np.sqrt(n) * np.eye(n))
    X = block_inverse(A, base=128)
    want = torch.linalg.inv(A)
    assert (X - want).abs().max() <= 1e-12 * want.abs().max()


def test_pivot_inverse_routes(monkeypatch):
    """pivot_inverse: the block route accepts an accurate inverse, refines a slightly wrong one by one
    Newton step, and falls back to the pivoted LU when a leading block is singular (no pivoting across
    the recursion's split)."""
    from sem_amd import linalg
    monkeypatch.setattr(VS, "_PIVOT_INV", "block")
    r = np.random.default_rng(12)
    n = 600
    A = torch.as_tensor(r.uniform(-1, 1, (n, n)) + 4 * np.sqrt(n) * np.eye(n))
    want = torch.linalg.inv(A)
    X = VS.pivot_inverse(A)
    assert (X - want).abs().max() <= 1e-12 * want.abs().max()
    # a perturbed block inverse: E = A X - I is a contraction, one Newton step squares it
    real = linalg.block_inverse
    monkeypatch.setattr(linalg, "block_inverse", lambda a, base=256, out=None: real(a) * (1 + 1e-7))
    X = VS.pivot_inverse(A)
    assert (X - want).abs().max() <= 1e-11 * want.abs().max()
    monkeypatch.setattr(linalg, "block_inverse", real)
    # leading block exactly singular: the recursion yields non-finite entries, the LU route takes over
    Z = torch.zeros((n, n), dtype=torch.float64)
    Z[: n // 2, n // 2:] = torch.eye(n - n // 2, dtype=torch.float64)[: n // 2]
    Z[n // 2:, : n // 2] = torch.eye(n // 2, dtype=torch.float64)[: n - n // 2]
    Z += torch.as_tensor(r.uniform(-1e-3, 1e-3, (n, n))) * torch.as_tensor(np.kron(
        np.array([[0.0, 1.0], [1.0, 1.0]]), np.ones((n // 2, n // 2))))
    X = VS.pivot_inverse(Z)
    E = Z @ X - torch.eye(n, dtype=torch.float64)
    assert E.abs().max() <= 1e-10
