"""CPU tests of the nested-dissection velocity solve (sem_amd/solvers/nested_dissection.py): the element shares
sum to the oracle's assembled velocity Jacobian (NavierStokes_Solver.py:123-136,176-183) on every non-Dirichlet
row, the dissection eliminates every unknown exactly once, and the torch path of the solve reproduces SciPy's
sparse solve of the Dirichlet-row-replaced Jacobian (the reference's `splu`, :184-192)."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla
import torch

from velocity_blocks import oracle_velocity_jacobian
from sem_amd.solvers.nested_dissection import NDTree, NestedDissectionSolver, _gll_tables, element_matrices

CASES = [(4, 3, 2, 100.0), (2, 2, 3, 400.0), (6, 2, 2, 1000.0), (3, 1, 1, 1.0), (2, 7, 2, 300.0), (3, 6, 5, 50.0),
         (4, 1, 3, 20.0), (5, 3, 7, 150.0)]


def _kw(ns, u, v, Re):
    t = torch.as_tensor
    return dict(c_stiff=1.0, c_gradx=Re, cu=t(u), c_grady=Re, cv=t(v), juu=t(Re * (ns.Gx @ u)),
                jvv=t(Re * (ns.Gy @ v)), juv=t(Re * (ns.Gy @ u)), jvu=t(Re * (ns.Gx @ v)))


def _oracle_index(t, flat):
    """Line-array flat index -> the oracle's [u | v] index (component-major, x-major nodes)."""
    gx, r = np.divmod(flat, t.m)
    c, gy = np.divmod(r, t.NY)
    return c * (t.NX * t.NY) + gx * t.NY + gy


@pytest.mark.parametrize("P,nex,ney,Re", CASES)
def test_element_shares_sum_to_the_jacobian(P, nex, ney, Re):
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    J = ns.Jvelo.toarray()
    t = NDTree(P, nex, ney, 2)
    A = element_matrices(t, np.arange(nex * ney), 1.0 / nex, 1.0 / ney, *_gll_tables(P), **_kw(ns, u, v, Re)).numpy()
    S = np.zeros_like(J)
    for e in range(nex * ney):
        g = _oracle_index(t, t.eflat[e])
        S[np.ix_(g, g)] += A[e]
    D = np.zeros(J.shape[0], dtype=bool)
    D[_oracle_index(t, t.eflat.reshape(-1))] = t.eD.reshape(-1)
    assert np.array_equal(D, np.concatenate((ns.mask_bound, ns.mask_bound)))
    assert np.abs(S[~D] - J[~D]).max() <= 1e-14 * np.abs(J).max()
    assert not S[D].any()


@pytest.mark.parametrize("P,nex,ney", [(3, 5, 3), (2, 8, 8), (4, 7, 2), (2, 1, 6), (5, 9, 4)])
def test_dissection_eliminates_every_unknown_once(P, nex, ney):
    t = NDTree(P, nex, ney, 2)
    owned = [t.eflat[:, :t.ni].reshape(-1)] + [f["S"] for f in t.fronts]
    allv = np.concatenate(owned)
    assert len(np.unique(allv)) == len(allv)
    nonD = np.unique(t.eflat[~t.eD])
    assert np.array_equal(np.sort(allv), nonD)
    for f in t.fronts:   # a front's boundary: ancestor-separator nodes only, never Dirichlet
        assert not np.isin(f["B"], t.eflat[t.eD]).any()
    for f in t.fronts:   # binary: two children, each update fully inside the front
        assert len(f["maps"]) == 2
        for (kind, cid), pos in zip(f["children"], f["maps"]):
            assert (pos >= 0).all() or kind == "e"


@pytest.mark.parametrize("P,nex,ney,Re", CASES)
def test_nd_solve_matches_sparse_lu(P, nex, ney, Re):
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    vs = NestedDissectionSolver(P, nex, ney, "cpu")
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, **_kw(ns, u, v, Re))
    r = np.random.default_rng(5)
    bu, bv = r.uniform(-1, 1, ns.N), r.uniform(-1, 1, ns.N)
    xu, xv = vs.solve(torch.as_tensor(bu), torch.as_tensor(bv))
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu, bv)))
    got = np.hstack((xu.numpy(), xv.numpy()))
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()


@pytest.mark.parametrize("P,nex,ney,Re,smooth,split", [
    (4, 3, 2, 100.0, 0.3, True), (8, 2, 3, 1000.0, 0.3, True), (10, 2, 2, 1000.0, 0.3, True),
    (12, 2, 2, 1000.0, 0.3, True), (5, 3, 7, 150.0, 0.0, False), (12, 2, 3, 200.0, 0.0, False)])
def test_nd_split_leaves(P, nex, ney, Re, smooth, split):
    """The split leaves (A_uu^-1, S_v^-1 and the diagonal Newton couplings instead of A_ii^-1: half the leaf bytes)
    are taken on smooth velocity fields and refused, by the factor's per-element probe, where the coupling rivals
    the stiffness (random fields); either way the solve is SciPy's.  The split V_e and the forward step agree with
    the dense elimination."""
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex, smooth=smooth)
    vs = NestedDissectionSolver(P, nex, ney, "cpu")
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, **_kw(ns, u, v, Re))
    assert vs.split == split and (vs._leafB is not None) == split and (vs._leafF is None) == split
    assert vs.split_eta is not None and (vs.split_eta <= vs.SPLIT_ETA) == split
    assert sum(st[0] == "leaf" for st in vs._steps) == int(split)
    r = np.random.default_rng(5)
    bu, bv = r.uniform(-1, 1, ns.N), r.uniform(-1, 1, ns.N)
    xu, xv = vs.solve(torch.as_tensor(bu), torch.as_tensor(bv))
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu, bv)))
    got = np.hstack((xu.numpy(), xv.numpy()))
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()
    n = (P - 1) ** 2
    ld = n + (n & 1)
    leaf = (2 * n * ld + 2 * ld) if split else 4 * n * n
    t = vs.tree
    assert vs.bytes_per_solve() - t.bytes_per_solve(not split) == 8 * nex * ney * (leaf - ((4 * n * n) if split else
                                                                                          2 * n * ld + 2 * ld))


def test_nd_split_refused_when_a_component_block_is_singular():
    """A_uu singular while A_ii is not (the components coupled only through juv = jvu = 1: J swaps u and v off the
    Dirichlet rows): the split leaves' inverse fails, the factor takes Xi instead, and the solve is exact."""
    P, nex, ney = 3, 3, 2
    vs = NestedDissectionSolver(P, nex, ney, "cpu")
    N = vs.NX * (ney * P + 1)
    one = torch.ones(N, dtype=torch.float64)
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, juv=one, jvu=one)
    assert not vs.split and vs.split_eta == float("inf") and vs._leafF is not None
    r = np.random.default_rng(2)
    bu, bv = torch.as_tensor(r.uniform(-1, 1, N)), torch.as_tensor(r.uniform(-1, 1, N))
    xu, xv = vs.solve(bu, bv)
    x, y = np.divmod(np.arange(N), ney * P + 1)
    D = (x == 0) | (x == vs.NX - 1) | (y == 0) | (y == ney * P)
    assert torch.equal(xu[D], bu[D]) and torch.equal(xv[D], bv[D])
    assert (xu[~D] - bv[~D]).abs().max() <= 1e-14 and (xv[~D] - bu[~D]).abs().max() <= 1e-14


def test_nd_refuses_other_dirichlet_sets():
    vs = NestedDissectionSolver(3, 2, 2, "cpu")
    with pytest.raises(ValueError):
        vs.factor_coeffs(0.5, 0.5, c_stiff=1.0, dir_sides=1 | 2)
    with pytest.raises(ValueError):
        NestedDissectionSolver(1, 2, 2, "cpu")


def test_launch_policy():
    """sem_front_gemv's per-launch choices: lanes per row by the median row length (64 for rows of >= 192 doubles),
    the wide tile unless the launch would have fewer than 256 workgroups, and the column form only for forward front
    levels with rows of <= 128 doubles."""
    S = NestedDissectionSolver
    assert S._launch_shape(np.array([242] * 4), np.array([338] * 4)) == (64, 4)
    assert S._launch_shape(np.array([242] * 20000), np.array([242] * 20000)) == (64, 16)
    assert S._launch_shape(np.array([96] * 4), np.array([242] * 4)) == (16, 16)
    assert S._launch_shape(np.array([22] * 4), np.array([174] * 4)) == (4, 64)
    assert S._launch_shape(np.array([3070] * 2), np.array([5000] * 2)) == (64, 16)   # 626 wide tiles
    assert S._launch_shape(np.array([3070]), np.array([3070])) == (64, 4)            # the root: 192
    vs = S.__new__(S)
    assert vs._launch_form(False, 8192, np.array([22] * 8192), False) == 1
    assert vs._launch_form(True, 8192, np.array([22] * 8192), False) == 0
    assert vs._launch_form(False, 16384, np.array([242] * 16384), True) == 0
    assert vs._launch_form(False, 1, np.array([3070]), False) == 0
    assert vs._launch_form(False, 1024, np.array([92] * 1024), False) == 1
    assert vs._launch_form(False, 256, np.array([180] * 256), False) == 0
    vs.forms = "rows"
    assert vs._launch_form(False, 8192, np.array([22] * 8192), False) == 0
