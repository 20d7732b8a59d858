"""CPU tests of the velocity-Jacobian static condensation (sem_amd/solvers/velocity_solve.py):
the pieces describe the oracle's Dirichlet-row-replaced Jacobian exactly (the line-coupling
structure the condensation relies on), and the condensed solve reproduces SciPy's sparse solve of
the same matrix (the reference uses SuperLU on it, NavierStokes_Solver.py:176-192)."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla
import torch

from velocity_blocks import assemble, extract, oracle_cd_jacobian, oracle_velocity_jacobian
from sem_amd.solvers.velocity_solve import VelocityJacobianSolver

CASES = [(4, 3, 2, 100.0), (2, 2, 3, 400.0), (1, 4, 3, 10.0), (6, 2, 2, 1000.0), (3, 1, 1, 1.0), (2, 7, 2, 300.0),
         (3, 6, 2, 50.0)]


@pytest.mark.parametrize("P,nex,ney,Re", CASES)
def test_pieces_describe_the_jacobian_exactly(P, nex, ney, Re):
    ns, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    J = ns.Jvelo.toarray()
    assert np.array_equal(assemble(extract(J, P, nex, ney), P, nex, ney), J)


@pytest.mark.parametrize("P,nex,ney,Re", CASES)
@pytest.mark.parametrize("interior,sweep", [("nested", "cr"), ("nested", "thomas"), ("lu", "cr"), ("inverse", "thomas")])
def test_condensed_solve_matches_sparse_lu(P, nex, ney, Re, interior, sweep):
    ns, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    pcs = {k: torch.as_tensor(v) for k, v in extract(ns.Jvelo.toarray(), P, nex, ney).items()}
    vs = VelocityJacobianSolver(P, nex, ney, "cpu", interior=interior, sweep=sweep)
    vs.factor(pcs.get("AII"), pcs["D"], pcs.get("aIB"), pcs.get("aBI"), pcs["E"], pcs["F"])
    r = np.random.default_rng(5)
    bu, bv = r.uniform(-1, 1, ns.N), r.uniform(-1, 1, ns.N)
    xu, xv = vs.solve(torch.as_tensor(bu), torch.as_tensor(bv))
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu, bv)))
    got = np.hstack((xu.numpy(), xv.numpy()))
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()
    # and it is a solve of J: small residual relative to |J||x|
    J = ns.Jvelo
    res = J @ got - np.hstack((bu, bv))
    assert np.abs(res).max() <= 1e-11 * (abs(J).max() * np.abs(got).max())


@pytest.mark.parametrize("P,nex,ney,Pe", [(4, 3, 2, 40.0), (8, 2, 3, 710.0), (1, 4, 3, 10.0), (3, 1, 1, 1.0)])
@pytest.mark.parametrize("sweep", ["cr", "thomas"])
def test_scalar_condensation_solves_the_cd_jacobian(P, nex, ney, Pe, sweep):
    """ncomp=1: the convection-diffusion Jacobian (the CD solver's preconditioner) condenses the
    same way, and the condensed solve reproduces SciPy's sparse solve."""
    cd, A, _, _ = oracle_cd_jacobian(P, nex, ney, Pe, seed=P + nex)
    Ad = A.toarray()
    pcs = extract(Ad, P, nex, ney, ncomp=1)
    assert np.array_equal(assemble(pcs, P, nex, ney, ncomp=1), Ad)
    pcs = {k: torch.as_tensor(v) for k, v in pcs.items()}
    vs = VelocityJacobianSolver(P, nex, ney, "cpu", sweep=sweep, ncomp=1)
    vs.factor(pcs.get("AII"), pcs["D"], pcs.get("aIB"), pcs.get("aBI"), pcs["E"], pcs["F"])
    b = np.random.default_rng(7).uniform(-1, 1, cd.N)
    got = vs.solve1(torch.as_tensor(b)).numpy()
    want = spla.spsolve(A.tocsc(), b)
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()
    with pytest.raises(ValueError):
        vs.solve(torch.as_tensor(b), torch.as_tensor(b))


@pytest.mark.parametrize("P,nex,ney,Re", [(4, 5, 2, 100.0), (3, 6, 2, 50.0), (6, 3, 2, 1000.0), (5, 4, 7, 400.0)])
@pytest.mark.parametrize("chunk_cols", [1, 2])
@pytest.mark.parametrize("edge", ["dense", "blocklu", "thomas"])
def test_condensed_chunked_factor_matches_sparse_lu(P, nex, ney, Re, chunk_cols, edge):
    """factor_condensed (the ABI-7 path: the condensed pieces of chunk_cols element columns at a time,
    sem_condensed_blocks' col_begin/col_end contract) solves the Jacobian; the edge Schur blocks inverted
    densely or by the checked block LU of their block-tridiagonal form, or (ABI 9) kept as the block-Thomas
    factors that block LU produced and solved by forward / back sweeps."""
    ns, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    pcs = {k: torch.as_tensor(v) for k, v in extract(ns.Jvelo.toarray(), P, nex, ney).items()}
    ch = VelocityJacobianSolver(P, nex, ney, "cpu")
    cond = ch.condense_dense(pcs["AII"])

    def fill(blocks, cols):   # the kernel's contract: condensed pieces of columns cols, line pieces in full
        c0, c1 = cols
        for k in ("D", "aIB", "aBI", "E", "F"):
            blocks[k].copy_(pcs[k])
        for k, v in cond.items():
            blocks[k].copy_(v[c0:c1])

    if edge in ("blocklu", "thomas"):
        ch.edge_dense_max = 0
    ch.edge_solve = "thomas" if edge == "thomas" else "dense"
    ch.factor_condensed(fill, chunk_cols=chunk_cols)
    assert ch._edge_thomas == (edge == "thomas")
    r = np.random.default_rng(9)
    bu, bv = (torch.as_tensor(r.uniform(-1, 1, ns.N)) for _ in range(2))
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu.numpy(), bv.numpy())))
    got = np.hstack([t.numpy() for t in ch.solve(bu, bv)])
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()


@pytest.mark.parametrize("nb,b,seed", [(1, 3, 0), (2, 5, 1), (9, 4, 2), (30, 6, 3)])
def test_block_tridiagonal_inverse(nb, b, seed):
    """_blocktri_inverse (block LU with pivoted pivot-block inverses, then block Thomas against I) equals the
    dense inverse; a column that needs inter-block pivoting (a singular leading block) is detected by the
    residual check and inverted densely."""
    r = np.random.default_rng(seed)
    cc = 3
    Sd = torch.as_tensor(r.uniform(-1, 1, (cc, nb, b, b)) + 4 * b * np.eye(b))
    Su = torch.as_tensor(r.uniform(-1, 1, (cc, nb - 1, b, b)))
    Sl = torch.as_tensor(r.uniform(-1, 1, (cc, nb - 1, b, b)))
    if nb > 1:
        Sd[1, 0] = 0.0   # zero first pivot block: the block LU fails, the dense pivoted inverse does not
        Su[1, 0] = torch.eye(b, dtype=torch.float64) * 3
        Sl[1, 0] = torch.eye(b, dtype=torch.float64) * 2
    vs = VelocityJacobianSolver(2, 1, 1, "cpu")
    vs.edge_dense_max = 0
    X = vs._blocktri_inverse(Sd, Su, Sl)
    S = VelocityJacobianSolver._blocktri_dense(Sd, Su, Sl)
    want = torch.linalg.inv(S)
    assert torch.allclose(X, want, rtol=0, atol=1e-10 * want.abs().max().item())


def test_edge_thomas_falls_back_to_dense_inverses():
    """A column whose block LU fails the residual check (zero leading pivot block) switches the block-Thomas
    edge form to dense inverses: the columns factored before it get their inverses rebuilt from their
    factors, and the solve still reproduces SciPy's."""
    P, nex, ney, Re = 4, 4, 3, 100.0
    ns, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=5)
    pcs = {k: torch.as_tensor(v) for k, v in extract(ns.Jvelo.toarray(), P, nex, ney).items()}
    ch = VelocityJacobianSolver(P, nex, ney, "cpu")
    ch.edge_dense_max, ch.edge_solve = 0, "thomas"
    cond = ch.condense_dense(pcs["AII"])
    orig = VelocityJacobianSolver._blocktri_inverse

    def failing(self, Sd, Su, Sl, factors=False):   # pretend column 2's block LU failed its check
        X, fac = orig(self, Sd, Su, Sl, factors=True)
        return (X, None if self._c0 <= 2 < self._c0 + Sd.shape[0] else fac) if factors else X

    def fill(blocks, cols):
        ch._c0 = cols[0]
        for k in ("D", "aIB", "aBI", "E", "F"):
            blocks[k].copy_(pcs[k])
        for k, v in cond.items():
            blocks[k].copy_(v[cols[0]:cols[1]])

    VelocityJacobianSolver._blocktri_inverse = failing
    try:
        ch.factor_condensed(fill, chunk_cols=1)
    finally:
        VelocityJacobianSolver._blocktri_inverse = orig
    assert not ch._edge_thomas and ch._Se_inv is not None
    r = np.random.default_rng(2)
    bu, bv = (torch.as_tensor(r.uniform(-1, 1, ns.N)) for _ in range(2))
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu.numpy(), bv.numpy())))
    got = np.hstack([t.numpy() for t in ch.solve(bu, bv)])
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()


@pytest.mark.parametrize("n,m", [(3, 5), (4, 7), (5, 4), (9, 6), (12, 3), (13, 8)])
def test_twisted_thomas_matches_dense_solve(n, m):
    """The two-ended block-Thomas sweep (twisted_thomas_operators / twisted_thomas_solve: chains from line 0 and
    from line n-1 meeting at n // 2, odd and even line counts) against a dense solve of the assembled
    block-tridiagonal system, and against the one-ended fused sweep."""
    from sem_amd.solvers.velocity_solve import (fused_thomas_operators, fused_thomas_solve, twisted_thomas_operators,
                                                twisted_thomas_solve)
    g = torch.Generator().manual_seed(n * 100 + m)
    f64 = torch.float64
    Sd = torch.rand((n, m, m), dtype=f64, generator=g) - 0.5 + 3 * m * torch.eye(m, dtype=f64)
    Su = torch.rand((n - 1, m, m), dtype=f64, generator=g) - 0.5
    Sl = torch.rand((n - 1, m, m), dtype=f64, generator=g) - 0.5
    A = torch.zeros((n * m, n * m), dtype=f64)
    for L in range(n):
        A[L * m:(L + 1) * m, L * m:(L + 1) * m] = Sd[L]
        if L < n - 1:
            A[L * m:(L + 1) * m, (L + 1) * m:(L + 2) * m] = Su[L]
            A[(L + 1) * m:(L + 2) * m, L * m:(L + 1) * m] = Sl[L]
    rhs = torch.rand((n, m), dtype=f64, generator=g) - 0.5
    want = torch.linalg.solve(A, rhs.reshape(-1)).reshape(n, m)
    got = twisted_thomas_solve(twisted_thomas_operators(Sd, Su, Sl), rhs)
    assert (got - want).abs().max().item() <= 1e-12 * want.abs().max().item()
    # block right-hand sides (the strip solve's coupling solutions X0, X1 from the twisted factors)
    from sem_amd.solvers.velocity_solve import twisted_thomas_solve_mat
    Rm = torch.rand((n, m, 3), dtype=f64, generator=g) - 0.5
    wantm = torch.linalg.solve(A, Rm.reshape(n * m, 3)).reshape(n, m, 3)
    gotm = twisted_thomas_solve_mat(twisted_thomas_operators(Sd, Su, Sl), Rm)
    assert (gotm - wantm).abs().max().item() <= 1e-12 * wantm.abs().max().item()
    # the one-ended sweep's operators from the same blocks
    Dinv = torch.empty_like(Sd)
    Uh = torch.empty_like(Su)
    Dt = Sd[0]
    for L in range(n):
        if L > 0:
            Dt = Sd[L] - Sl[L - 1] @ Uh[L - 1]
        Dinv[L] = torch.linalg.inv(Dt)
        if L < n - 1:
            Uh[L] = Dinv[L] @ Su[L]
    one = fused_thomas_solve(*fused_thomas_operators(Dinv, Sl, Uh), rhs)
    assert (got - one).abs().max().item() <= 1e-12 * want.abs().max().item()


def test_refinement_gate_rejects_a_non_finite_factor():
    """a singular or overflowing factor makes the probe's backward error NaN, and max(0, nan) is 0 in
    Python -- the gate must raise instead of reading it as "no refinement needed".  (A singular interior block is
    caught earlier, by the factor's own inverse check; the probe's last line of defence is exercised with an
    operator that returns NaN.)"""
    P, nex, ney, Re = 4, 3, 2, 100.0
    ns, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    pcs = {k: torch.as_tensor(v) for k, v in extract(ns.Jvelo.toarray(), P, nex, ney).items()}
    J = ns.Jvelo
    NX = nex * P + 1

    def apply_lines(X):
        X3 = X.view(NX, 2, -1)
        y = J @ np.hstack((X3[:, 0].reshape(-1).numpy(), X3[:, 1].reshape(-1).numpy()))
        Y = torch.as_tensor(y).view(2, NX, -1)
        return torch.stack((Y[0], Y[1]), dim=1).reshape(X.shape)

    vs = VelocityJacobianSolver(P, nex, ney, "cpu", interior="inverse", sweep="thomas")
    vs.factor(pcs["AII"], pcs["D"], pcs["aIB"], pcs["aBI"], pcs["E"], pcs["F"])
    vs.set_operator(apply_lines)
    assert vs.check_refinement() < 1e-13               # the healthy factor passes
    A = pcs["AII"].clone()
    A[1] = 0.0
    with pytest.raises(RuntimeError):                   # a singular interior block: refused at factor time
        VelocityJacobianSolver(P, nex, ney, "cpu", interior="inverse", sweep="thomas").factor(
            A, pcs["D"], pcs["aIB"], pcs["aBI"], pcs["E"], pcs["F"])
    vs.set_operator(lambda X: apply_lines(X) * float("nan"))
    with pytest.raises(RuntimeError, match="non-finite"):
        vs.check_refinement()
