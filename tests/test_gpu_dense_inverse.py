"""GPU parity of the small dense inverse (sem_dense_inverse_small, sem_amd/csrc/dense_inverse.hip) and of
the GEMM-recursive pivot inverse built on it (sem_amd/linalg.py block_inverse), against torch's pivoted
LU inverse: leaves of every size class, strided views, blocks that need row pivoting, a singular block,
and whole pivot-sized blocks through velocity_solve.pivot_inverse."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel_res(A, X):
    E = A @ X - torch.eye(A.shape[-1], dtype=A.dtype, device=A.device)
    return (E.abs().max() / (A.abs().max() * X.abs().max())).item()


@pytest.mark.parametrize("n", [1, 2, 5, 16, 17, 33, 48, 63, 64])
def test_small_inverse_sizes(gpu, n):
    from sem_amd.linalg import small_inverse_into
    g = torch.Generator(device="cuda").manual_seed(n)
    A = torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
    A += n ** 0.5 * torch.eye(n, dtype=torch.float64, device="cuda")
    X = torch.full_like(A, float("nan"))
    small_inverse_into(A, X)
    want = torch.linalg.inv(A)
    assert (X - want).abs().max().item() <= 1e-12 * want.abs().max().item()


def test_small_inverse_views_and_pivoting(gpu):
    """Row-major views with a leading dimension in and out, and a block whose diagonal is zero (a
    permutation plus noise): without row pivoting the first step divides by zero."""
    from sem_amd.linalg import small_inverse_into
    n = 61
    g = torch.Generator(device="cuda").manual_seed(3)
    Pm = torch.zeros((n, n), dtype=torch.float64, device="cuda")
    Pm[torch.arange(n), (torch.arange(n) + 1) % n] = 1.0     # cyclic shift: regular, zero diagonal
    big = torch.zeros((n + 7, n + 11), dtype=torch.float64, device="cuda")
    big[3:3 + n, 5:5 + n] = Pm + 1e-3 * torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g)
    A = big[3:3 + n, 5:5 + n]
    out = torch.zeros((n + 2, 2 * n), dtype=torch.float64, device="cuda")
    X = out[1:1 + n, n // 2:n // 2 + n]
    small_inverse_into(A, X)
    assert _rel_res(A, X) < 1e-13
    assert out[0].abs().max().item() == 0.0 and out[:, :n // 2].abs().max().item() == 0.0   # nothing outside X


def test_small_inverse_pivots_tiny_scaled_blocks(gpu):
    """A block that needs row pivoting, scaled to 1e-300: the pivot key comes from the double itself, so
    magnitudes far below the float range still order the rows."""
    from sem_amd.linalg import small_inverse_into
    n = 40
    g = torch.Generator(device="cuda").manual_seed(5)
    Pm = torch.zeros((n, n), dtype=torch.float64, device="cuda")
    Pm[torch.arange(n), (torch.arange(n) + 1) % n] = 1.0
    A = 1e-300 * (Pm + 1e-3 * torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g))
    X = torch.zeros_like(A)
    small_inverse_into(A, X)
    assert torch.isfinite(X).all().item()
    assert _rel_res(A, X) < 1e-13


def test_small_inverse_singular_is_non_finite(gpu):
    from sem_amd.linalg import small_inverse_into
    A = torch.ones((8, 8), dtype=torch.float64, device="cuda")
    X = torch.zeros_like(A)
    small_inverse_into(A, X)
    assert not torch.isfinite(X).all().item()


@pytest.mark.parametrize("n,base", [(700, 64), (1541, 64), (1541, 128)])
def test_block_inverse_matches_lu(gpu, n, base):
    from sem_amd.linalg import block_inverse
    g = torch.Generator(device="cuda").manual_seed(n)
    A = torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) - 0.5
    A += 2 * n ** 0.5 * torch.eye(n, dtype=torch.float64, device="cuda")
    X = block_inverse(A, base=base)
    want = torch.linalg.inv(A)
    assert (X - want).abs().max().item() <= 1e-12 * want.abs().max().item()


def test_pivot_inverse_falls_back_when_a_leading_block_is_singular(gpu):
    from sem_amd.solvers import velocity_solve as VS
    n = 600
    g = torch.Generator(device="cuda").manual_seed(9)
    Z = torch.rand((n, n), dtype=torch.float64, device="cuda", generator=g) * 1e-3
    Z[: n // 2, : n // 2] = 0.0
    Z[: n // 2, n // 2:] += torch.eye(n // 2, dtype=torch.float64, device="cuda")
    Z[n // 2:, : n // 2] += torch.eye(n // 2, dtype=torch.float64, device="cuda")
    X = VS.pivot_inverse(Z)
    assert _rel_res(Z, X) < 1e-12
