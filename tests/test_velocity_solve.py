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


@pytest.mark.parametrize("P,nex,ney,Re", [(4, 5, 2, 100.0), (3, 6, 2, 50.0), (6, 3, 2, 1000.0)])
@pytest.mark.parametrize("chunk_cols", [1, 2])
def test_column_chunked_factor_matches_one_shot(P, nex, ney, Re, chunk_cols):
    """factor_from with a budget of chunk_cols columns (the cfg5 path: dense interiors assembled,
    condensed and freed a chunk at a time, sem_velocity_blocks' col_begin/col_end) gives the solve of
    the one-shot factorisation."""
    ns, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    pcs = {k: torch.as_tensor(v) for k, v in extract(ns.Jvelo.toarray(), P, nex, ney).items()}

    def fill(blocks, cols):   # the kernel's contract: A_II of columns cols, every other piece in full
        c0, c1 = cols
        for k in ("D", "aIB", "aBI", "E", "F"):
            blocks[k].copy_(pcs[k])
        blocks["AII"].copy_(pcs["AII"][c0:c1])

    one = VelocityJacobianSolver(P, nex, ney, "cpu")
    one.factor(pcs["AII"].clone(), pcs["D"], pcs["aIB"], pcs["aBI"], pcs["E"], pcs["F"])
    ch = VelocityJacobianSolver(P, nex, ney, "cpu")
    nI, m = ch.nI, ch.m
    ch.factor_from(fill, budget_bytes=chunk_cols * (nI * nI * 8 + 3 * nI * 2 * m * 8))
    r = np.random.default_rng(9)
    bu, bv = (torch.as_tensor(r.uniform(-1, 1, ns.N)) for _ in range(2))
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu.numpy(), bv.numpy())))
    for s in (ch, one):   # the same factor up to the summation order of the interface blocks
        got = np.hstack([t.numpy() for t in s.solve(bu, bv)])
        assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()
