"""GPU tests of the nested-dissection velocity solve (sem_amd/solvers/nested_dissection.py, HIP steps
sem_front_gemv / sem_front_scatter): the solve of the oracle's Dirichlet-row-replaced velocity Jacobian
(NavierStokes_Solver.py:176-192) against SciPy's sparse solve of the same matrix, bitwise graph replay against the
eager solve, agreement with the torch path of the same factors, and the factor's backward-error probe."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla
import torch

from velocity_blocks import oracle_velocity_jacobian

pytestmark = pytest.mark.gpu

CASES = [(4, 3, 2, 100.0), (2, 2, 3, 400.0), (6, 2, 2, 1000.0), (3, 1, 1, 1.0), (2, 7, 2, 300.0), (3, 6, 5, 50.0),
         (8, 5, 4, 1000.0), (12, 4, 6, 200.0), (16, 2, 3, 300.0)]


def _apply_lines(J, vs, dev):
    """J X on the solver's (NX, 2 NY) line arrays, through SciPy (the refinement gate's operator)."""
    N = J.shape[0] // 2

    def apply(X):
        x = torch.cat((X.view(vs.NX, 2, -1)[:, 0].reshape(-1), X.view(vs.NX, 2, -1)[:, 1].reshape(-1))).cpu().numpy()
        y = torch.as_tensor(J @ x, device=dev)
        return torch.stack((y[:N].view(vs.NX, -1), y[N:].view(vs.NX, -1)), 1).reshape(vs.NX, -1)
    return apply


def _kw(ns, u, v, Re, dev):
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)  # noqa: E731
    return dict(c_stiff=1.0, c_gradx=Re, cu=t(u), c_grady=Re, cv=t(v), juu=t(Re * (ns.Gx @ u)),
                jvv=t(Re * (ns.Gy @ v)), juv=t(Re * (ns.Gy @ u)), jvu=t(Re * (ns.Gx @ v)))


@pytest.mark.parametrize("P,nex,ney,Re", CASES)
def test_nd_solve_matches_sparse_lu(P, nex, ney, Re):
    from sem_amd.solvers.nested_dissection import NestedDissectionSolver
    dev = torch.device("cuda", 0)
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    vs = NestedDissectionSolver(P, nex, ney, dev)
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, **_kw(ns, u, v, Re, dev))
    vs.set_operator(_apply_lines(ns.Jvelo.tocsr(), vs, dev))
    eta0 = vs.check_refinement()     # one refinement step per solve when the factor's probe exceeds 1e-13
    r = np.random.default_rng(5)
    bu, bv = r.uniform(-1, 1, ns.N), r.uniform(-1, 1, ns.N)
    xu, xv = vs.solve(torch.as_tensor(bu, device=dev), torch.as_tensor(bv, device=dev))
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu, bv)))
    got = np.hstack((xu.cpu().numpy(), xv.cpu().numpy()))
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()
    J = ns.Jvelo
    res = J @ got - np.hstack((bu, bv))
    eta = np.abs(res).max() / (abs(J).sum(axis=1).max() * np.abs(got).max() + max(np.abs(bu).max(), np.abs(bv).max()))
    assert eta <= (1e-15 if vs.refine else 1e-13), (eta0, eta)
    if vs.refine:    # the refinement step's operator here is SciPy's (host): not capturable
        return
    # graph replay is the eager solve, bit for bit
    B = torch.stack((torch.as_tensor(bu, device=dev).view(vs.NX, -1), torch.as_tensor(bv, device=dev).view(vs.NX, -1)),
                    1).reshape(vs.NX, -1)
    xe = vs._solve_lines(B.clone())
    assert vs.capture()
    gu, gv = vs.solve(torch.as_tensor(bu, device=dev), torch.as_tensor(bv, device=dev))
    assert torch.equal(gu, xe.view(vs.NX, 2, -1)[:, 0].reshape(-1))
    assert torch.equal(gv, xe.view(vs.NX, 2, -1)[:, 1].reshape(-1))


def test_nd_hip_steps_match_the_torch_path():
    """The HIP launches and the per-front torch loop over the same device factors: same values (the torch GEMVs
    sum in another order, so to rounding)."""
    from sem_amd.solvers.nested_dissection import NestedDissectionSolver
    dev = torch.device("cuda", 0)
    P, nex, ney, Re = 5, 4, 3, 300.0
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=3)
    vs = NestedDissectionSolver(P, nex, ney, dev)
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, **_kw(ns, u, v, Re, dev))
    B = torch.rand((vs.NX, vs.m), dtype=torch.float64, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    x_hip = vs._solve_lines_once(B.clone())      # the HIP steps
    dev_type = vs.device
    vs.device = torch.device("cpu")          # the torch loop (it reads the device tensors through the same tables)
    try:
        x_t = NestedDissectionSolver._solve_lines_once(vs, B.clone())
    finally:
        vs.device = dev_type
    assert (x_hip - x_t).abs().max() <= 1e-12 * x_t.abs().max()


def test_nd_refinement_gate_and_factor_size():
    """The factor's probe measures a finite backward error and the gate follows it; the operator bytes one solve
    reads are the tree's count."""
    from sem_amd.solvers.nested_dissection import NestedDissectionSolver
    dev = torch.device("cuda", 0)
    P, nex, ney, Re = 8, 6, 6, 1000.0
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=11)
    vs = NestedDissectionSolver(P, nex, ney, dev)
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, **_kw(ns, u, v, Re, dev))
    vs.set_operator(_apply_lines(ns.Jvelo.tocsr(), vs, dev))
    eta = vs.check_refinement()
    assert np.isfinite(eta) and eta < 1e-12 and vs.refine == (eta > 1e-13)
    ops = sum(T[q].numel() for st in vs._steps if st[0] != "leaf" for (T, q, *_rest) in st[1])
    ops += sum(st[3]["coef"].numel() for st in vs._steps if st[0] == "fwd" and st[3] is not None)
    ops += vs._leafB.numel() if vs.split else 0
    assert ops * 8 == vs.bytes_per_solve()


def test_nd_gemv_forms_agree():
    """sem_front_gemv's column form (transposed operators, a thread per row: the deepest forward levels) against
    form 0 everywhere on the same factor: the two sum each row in another order, so they agree to the rounding the
    levels carry; each is deterministic."""
    from sem_amd.solvers.nested_dissection import NestedDissectionSolver
    dev = torch.device("cuda", 0)
    P, nex, ney, Re = 6, 7, 5, 400.0
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=5)
    vs = NestedDissectionSolver(P, nex, ney, dev)
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, **_kw(ns, u, v, Re, dev))
    assert any(d.form == 1 for d, *_ in vs._hip)
    B = torch.rand((vs.NX, vs.m), dtype=torch.float64, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    x_auto = vs._solve_lines(B.clone())
    assert torch.equal(vs._solve_lines(B.clone()), x_auto)
    vs.forms = "rows"
    vs._hip = vs._hip_plan()
    assert all(d.form == 0 for d, *_ in vs._hip)
    x_rows = vs._solve_lines(B.clone())
    # the same factor applied with another summation order inside the deepest levels' rows: the difference is that
    # rounding carried through the dependent levels (2.8e-13 relative measured on this random Re = 400 Jacobian)
    assert (x_auto - x_rows).abs().max() <= 1e-11 * x_rows.abs().max()


@pytest.mark.parametrize("P,nex,ney,Re", [(2, 3, 2, 300.0), (3, 2, 3, 100.0), (4, 3, 2, 100.0), (8, 3, 4, 1000.0),
                                          (10, 2, 3, 500.0), (12, 4, 3, 1000.0)])
def test_nd_split_leaf_kernel(P, nex, ney, Re):
    """sem_leaf_forward (one workgroup per element: A_uu^-1 in registers across its two products, S_v^-1 streamed,
    y_i straight to the line array, the boundary rows to the stage) on smooth-field Jacobians, every register tile
    (RK = 1..4: P = 2, 3, 4, 8, 10, 12): the solve is SciPy's, the torch path of the same factor agrees to rounding,
    graph replay is the eager solve bit for bit."""
    from sem_amd.solvers.nested_dissection import NestedDissectionSolver
    dev = torch.device("cuda", 0)
    ns, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=P + nex, smooth=0.3)
    vs = NestedDissectionSolver(P, nex, ney, dev)
    vs.factor_coeffs(1.0 / nex, 1.0 / ney, **_kw(ns, u, v, Re, dev))
    assert vs.split, vs.split_eta
    r = np.random.default_rng(5)
    bu, bv = r.uniform(-1, 1, ns.N), r.uniform(-1, 1, ns.N)
    B = torch.stack((torch.as_tensor(bu, device=dev).view(vs.NX, -1), torch.as_tensor(bv, device=dev).view(vs.NX, -1)),
                    1).reshape(vs.NX, -1)
    x_hip = vs._solve_lines_once(B.clone())
    want = spla.spsolve(ns.Jvelo.tocsc(), np.hstack((bu, bv)))
    got = np.hstack((x_hip.view(vs.NX, 2, -1)[:, 0].reshape(-1).cpu().numpy(),
                     x_hip.view(vs.NX, 2, -1)[:, 1].reshape(-1).cpu().numpy()))
    assert np.abs(got - want).max() <= 1e-10 * np.abs(want).max()
    J = ns.Jvelo
    res = J @ got - np.hstack((bu, bv))
    eta = np.abs(res).max() / (abs(J).sum(axis=1).max() * np.abs(got).max() + max(np.abs(bu).max(), np.abs(bv).max()))
    assert eta <= 1e-13, eta      # the refinement gate's bound (check_refinement)
    dev_type = vs.device
    vs.device = torch.device("cpu")
    try:
        x_t = NestedDissectionSolver._solve_lines_once(vs, B.clone())
    finally:
        vs.device = dev_type
    # another summation order in every product, carried through the dependent levels: the forward error follows
    # the Jacobian's conditioning (4.5e-12 relative at P = 4, Re = 1000 on 3 x 2 elements), the backward error above
    # does not
    assert (x_hip - x_t).abs().max() <= 1e-10 * x_t.abs().max()
    assert vs.capture()
    gu, gv = vs.solve(torch.as_tensor(bu, device=dev), torch.as_tensor(bv, device=dev))
    assert torch.equal(gu, x_hip.view(vs.NX, 2, -1)[:, 0].reshape(-1))
    assert torch.equal(gv, x_hip.view(vs.NX, 2, -1)[:, 1].reshape(-1))
