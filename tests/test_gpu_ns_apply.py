"""GPU parity of the fused Navier-Stokes apply (sem_ns_apply, sem_amd/csrc/ns_apply.hip): the three
residuals (NavierStokes_Solver.py:93-121) and the three differentials (:138-160) in one launch each,
against the oracle's assembled-CSR restatement at random states -- including a mesh whose pinned
pressure node int(N/2) lies on the boundary (even NX, NY), where the two statement orders differ --
and the captured Schur-complement matvec against its definition through _get_dresiduals."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# (P, nex, ney, Re, Gr): the last one has NX = NY = 10, so the pin int(N/2) = 50 sits on y = 0
CASES = [(4, 3, 2, 100.0, 50.0), (1, 4, 3, 10.0, 0.0), (8, 4, 4, 1000.0, 20.0), (5, 2, 3, 250.0, 7.0),
         (3, 3, 3, 400.0, 30.0)]


def _state(N, seed):
    r = np.random.default_rng(seed)
    return [r.uniform(-1, 1, N) for _ in range(8)]


def _rel(a, b):
    return np.abs(np.asarray(a) - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(params=["band", "tile"])
def ns_kernel(request):
    """sem_ns_apply's two forms (SEM_TUNE_NS_APPLY): the band form (default) and the LDS-tile form."""
    from sem_amd import _lib
    lib = _lib.load()
    _lib.check(lib.sem_set_tuning(_lib.TUNE_NS_APPLY, 1 if request.param == "tile" else 0))
    yield request.param
    _lib.check(lib.sem_set_tuning(_lib.TUNE_NS_APPLY, 0))


@pytest.mark.parametrize("P,nex,ney,Re,Gr", CASES + [(12, 3, 5, 1000.0, 40.0), (16, 2, 2, 300.0, 5.0)])
def test_fused_residuals_match_oracle(gpu, ns_kernel, P, nex, ney, Re, Gr):
    from oracle import sem_oracle as O
    from sem_amd.solvers import NavierStokesSolver
    ref = O.NSOracle(1.0, 1.3, Re, Gr, P, nex, ney, u_N=1.0, v_W=0.25)
    ns = NavierStokesSolver(1.0, 1.3, Re, Gr, P, nex, ney, u_N=1.0, v_W=0.25, iprint=[])
    u, v, p, T, du, dv, dp, dT = _state(ns.N, P * 7 + nex)
    got = ns._get_residuals(u, v, p, T)
    want = ref.residuals(u, v, p, T)
    for a, b in zip(got, want):
        assert _rel(a, b) < 1e-13
    ref.calc_jacobians(u, v)
    ns._calc_jacobians(u, v)
    for t in (dT, None):
        got = ns._get_dresiduals(du, dv, dp, t)
        want = ref.dresiduals(du, dv, dp, t)
        for a, b in zip(got, want):
            assert _rel(a, b) < 1e-13


def test_pin_on_the_boundary_follows_the_statement_order(gpu):
    from oracle import sem_oracle as O
    from sem_amd.solvers import NavierStokesSolver
    ns = NavierStokesSolver(1.0, 1.0, 100.0, 0.0, 3, 3, 3, u_N=1.0, iprint=[])
    pin = int(ns.N / 2)
    assert ns._mask_bound[pin] and ns._pin == pin
    ref = O.NSOracle(1.0, 1.0, 100.0, 0.0, 3, 3, 3, u_N=1.0)
    u, v, p, T, du, dv, dp, _ = _state(ns.N, 5)
    rc = ns._get_residuals(u, v, p, T)[2]
    assert rc[pin] != p[pin] and abs(rc[pin] - ref.residuals(u, v, p, T)[2][pin]) < 1e-12  # Neumann row wins
    ns._calc_jacobians(u, v)
    ref.calc_jacobians(u, v)
    drc = ns._get_dresiduals(du, dv, dp)[2]
    assert drc[pin] == dp[pin]                                                              # pinned row wins


def test_one_launch_per_output_set(gpu, monkeypatch):
    """one fused launch per _get_residuals / _get_dresiduals, no sem_apply."""
    from sem_amd.solvers import NavierStokesSolver
    ns = NavierStokesSolver(1.0, 1.0, 100.0, 10.0, 4, 3, 3, u_N=1.0, iprint=[])
    m = ns._mesh
    calls = {"apply": 0, "ns_apply": 0}
    orig_apply, orig_ns = m.apply, m.ns_apply

    def count(name, f):
        def g(*a, **k):
            calls[name] += 1
            return f(*a, **k)
        return g
    monkeypatch.setattr(m, "apply", count("apply", orig_apply))
    monkeypatch.setattr(m, "ns_apply", count("ns_apply", orig_ns))
    u, v, p, T, du, dv, dp, dT = (m.to_device(a) for a in _state(ns.N, 1))
    ns._get_residuals(u, v, p, T)
    assert calls == {"apply": 0, "ns_apply": 1}
    ns._calc_jacobians(u, v)          # the four Jacobian diagonals Re G_x u, ... (4 gradient applies)
    calls.update(apply=0, ns_apply=0)
    ns._get_dresiduals(du, dv, dp, dT)
    assert calls == {"apply": 0, "ns_apply": 1}


@pytest.mark.parametrize("graph", [True, False])
def test_schur_matvec_matches_definition(gpu, graph):
    """S dp = dres_cont(-J^-1 [G_x dp; G_y dp]_D, dp) (NavierStokes_Solver.py:194-203)."""
    from sem_amd.solvers import NavierStokesSolver
    from sem_amd.solvers.navier_stokes import _SchurComplement
    ns = NavierStokesSolver(1.0, 1.0, 400.0, 0.0, 5, 4, 3, u_N=1.0, iprint=[])
    u, v, p, T, *_ = (ns._mesh.to_device(a) for a in _state(ns.N, 2))
    ns._get_residuals(u, v, p, T)
    ns._calc_jacobians(u, v)
    vs = ns._velocity_solver()
    S = _SchurComplement(ns, vs, graph=graph)
    assert (S._graph is not None) == graph
    Z = torch.zeros_like(u)
    for seed in range(3):
        dp = ns._mesh.to_device(np.random.default_rng(seed).uniform(-1, 1, ns.N))
        fx, fy = vs.solve(*ns._get_dresiduals(Z, Z, dp)[:2])
        want = ns._get_dresiduals(-fx, -fy, dp)[2]
        got = S(dp)
        assert torch.allclose(got, want, rtol=0, atol=1e-12 * want.abs().max().item())
