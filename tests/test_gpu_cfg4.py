"""BASELINE cfg4 in the GPU suite: Boussinesq_Sequential at Ra = 1e6 on 48 x 48 elements, P = 8, one
MI355X -- the coupler counterpart (sem_amd/solvers/boussinesq.py, OpenMDAO/Boussinesq_SequentialCoupler.py:
66-97) at full size, pinned by the oracle at the converged state of the device's Ra continuation
(tests/golden/cfg4_state.npz; the oracle side is tests/golden/make_oracle_fixtures.py cfg4, and the oracle
is also evaluated live here as the checker):

* the device coupled residual against the oracle's, at the state and at a seeded perturbation of it;
* ||R|| <= atol_nonlin at the state, on the device and for the oracle (the device solution solves the
  reference's discrete equations);
* one device NS _get_update (velocity condensation inside the Schur Krylov solve) and one CD _get_update
  (the condensed direct preconditioner inside GMRES) for seeded right-hand sides, through the oracle's
  _get_dresiduals, and the CD update against the oracle's exact solve;
* the midline maxima of the reference example (Examples/Boussinesq_Sequential_Example.py:20-40) by the
  device interpolation kernel, against de Vahl Davis (1983) and Le Quere (1991);
* the whole module within 60 s."""
import time

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

NE, P, RE, RA, PR = 48, 8, 1e3, 1e6, 0.71
_T0 = {}


def _rhs(N, seed=44):
    """Same draws as make_oracle_fixtures.cfg4_rhs: bT, then (bu, bv, bp)."""
    r = np.random.default_rng(seed)
    return r.uniform(-1, 1, N), tuple(r.uniform(-1, 1, N) for _ in range(3))


@pytest.fixture(scope="module")
def cfg4(gpu):
    _T0["t"] = time.perf_counter()
    from oracle import sem_oracle as O
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    c = BoussinesqCoupler(1.0, 1.0, RE, RA, PR, P, NE, NE, P, NE, NE, mode="JNK")
    x = golden("cfg4_state.npz")["x"]
    N = c.Nns
    T, u, v, p = x[:N], x[N:2 * N], x[2 * N:3 * N], x[3 * N:]
    cd = O.CDOracle(1.0, 1.0, RE * PR, P, NE, NE, T_W=0.5, T_E=-0.5)
    ns = O.NSOracle(1.0, 1.0, RE, RA / PR, P, NE, NE)
    return dict(c=c, x=x, N=N, T=T, u=u, v=v, p=p, cd=cd, ns=ns, fx=golden("cfg4_oracle.npz"))


def test_cfg4_coupled_residual_matches_oracle(cfg4):
    c, x, fx, N = cfg4["c"], cfg4["x"], cfg4["fx"], cfg4["N"]
    R = c.residuals(x)
    want = fx["R_sample"]
    idx = fx["sample_idx"]
    assert R.shape == (4 * N,) and int(fx["DOF"]) == c.DOF
    # converged: the residual is round-off of terms of order |Sys||x|; both sides agree far below atol
    assert np.abs(R[idx] - want).max() <= 1e-3 * c.atol_nonlin
    assert abs(np.linalg.norm(R) - float(fx["R_norm"])) <= 1e-3 * c.atol_nonlin
    # live oracle on the full vector at a seeded 10 % perturbation of the state, where R is of the order of
    # the operator terms (no cancellation to the converged round-off): the 1e-13 bar of SURVEY 8c
    o_cd, o_ns = cfg4["cd"], cfg4["ns"]
    r = np.random.default_rng(45)
    xp = x * (1.0 + 0.1 * r.uniform(-1, 1, x.size))
    Rp = c.residuals(xp)
    Tp, up, vp, pp = (xp[i * N:(i + 1) * N] for i in range(4))
    blocks = (o_cd.residuals(Tp, up, vp),) + tuple(o_ns.residuals(up, vp, pp, Tp))
    for i, b in enumerate(blocks):
        assert np.abs(Rp[i * N:(i + 1) * N] - b).max() <= 1e-13 * np.abs(b).max(), i


def test_cfg4_state_is_converged(cfg4):
    """||R||_2 <= mtol_nonlin sqrt(DOF) (Boussinesq_SequentialCoupler.py:61-63,80) on the device and for the
    oracle's residual (make_oracle_fixtures cfg4)."""
    c, x, fx = cfg4["c"], cfg4["x"], cfg4["fx"]
    assert np.linalg.norm(c.residuals(x)) <= c.atol_nonlin
    assert float(fx["R_norm"]) <= c.atol_nonlin


def test_cfg4_ns_update_solves_the_oracle_linearisation(cfg4):
    """One NS block-Jacobi solve (solve_linear, NavierStokes_Component.py:52-60 -> _get_update) at the
    state's linearisation, for the right-hand side the oracle's _get_dresiduals (NavierStokes_Solver.py:
    138-160) makes of a smooth seeded step (du, dv vanish on the walls): the device update reproduces
    the step's velocities (unique; the pressure is unique up to the spurious modes of the equal-order
    discretisation) and the oracle's _get_dresiduals of the update reproduces the
    right-hand side.  The device stops the Schur Krylov solve at the reference's rule
    ||r||_2 <= mtol sqrt(N) with the couplers' mtol_internal = 1e-13; the velocity rows are solved
    directly (residual ~1e-14 relative)."""
    c, x, N = cfg4["c"], cfg4["x"], cfg4["N"]
    o = cfg4["ns"]
    c.residuals(x)
    c.linearize(x)
    X, Y = o.points
    du = 1e-3 * np.sin(np.pi * X) * np.sin(2 * np.pi * Y)
    dv = -2e-3 * np.sin(2 * np.pi * X) * np.sin(np.pi * Y)
    dp = 1e-2 * np.cos(np.pi * X) * np.cos(np.pi * Y)
    o.residuals(cfg4["u"], cfg4["v"], cfg4["p"], cfg4["T"])
    o.calc_jacobians(cfg4["u"], cfg4["v"])
    bu, bv, bp = o.dresiduals(du, dv, dp)
    z = np.zeros(N)
    c.ns._progress = 500
    gu, gv, gp = c.ns._get_update(bu, bv, bp, du0=z, dv0=z, dp0=z)
    lin = o.dresiduals(np.asarray(gu), np.asarray(gv), np.asarray(gp))
    err = np.sqrt(sum(np.sum((a - b) ** 2) for a, b in zip(lin, (bu, bv, bp))))
    assert err <= 1e2 * 1e-13 * np.sqrt(N), err
    # velocities: to the accuracy the Schur stopping rule implies (measured 3.6e-6 relative)
    for a, b in ((gu, du), (gv, dv)):
        assert np.abs(np.asarray(a) - b).max() <= 2e-5 * np.abs(b).max()
    assert 0 < c.ns.schur_matvecs < 3000


def test_cfg4_cd_update_matches_oracle_solve(cfg4):
    """One CD block-Jacobi solve (ConvectionDiffusion_Component.py:51-57 -> _get_update) against the
    oracle's exact solve of the same linearised system, and through the oracle's _get_dresiduals."""
    c, x, N, fx = cfg4["c"], cfg4["x"], cfg4["N"], cfg4["fx"]
    o = cfg4["cd"]
    c.residuals(x)
    c.linearize(x)
    bT, _ = _rhs(N)
    dT = np.asarray(c.cd._get_update(bT, dT0=np.zeros(N)))
    o.residuals(cfg4["T"], cfg4["u"], cfg4["v"])
    res = np.linalg.norm(o.dresiduals(dT) - bT)
    assert res <= 10 * 1e-13 * np.sqrt(N), res
    want = fx["cd_update_sample"]
    assert np.abs(dT[::97] - want).max() <= 1e-9 * np.abs(want).max()
    assert abs(np.linalg.norm(dT) - float(fx["cd_update_norm"])) <= 1e-9 * float(fx["cd_update_norm"])


def test_cfg4_midline_maxima_de_vahl_davis(cfg4):
    """u_max Re Pr on x = 1/2 and v_max Re Pr on y = 1/2 by the device interpolation kernel
    (sem_eval_interpolation, SEM.py:248-273).  de Vahl Davis (1983), Ra = 1e6: 64.63 at y = 0.850 and
    219.36 at x = 0.0379; his Ra = 1e6 values are extrapolated from coarse meshes, and the later
    high-accuracy solution of Le Quere (1991) is 64.83 / 220.6.  The device state matches Le Quere to
    0.05 %, hence de Vahl Davis' u_max to 0.5 % and his v_max to 0.6 %."""
    c, u, v = cfg4["c"], cfg4["u"], cfg4["v"]
    s = np.linspace(0.0, 1.0, 2001)
    k = RE * PR
    um = np.asarray(c.ns._get_interpol(u, np.meshgrid([0.5], s, indexing="ij")))[0] * k
    vm = np.asarray(c.ns._get_interpol(v, np.meshgrid(s, [0.5], indexing="ij")))[:, 0] * k
    i, j = int(um.argmax()), int(vm.argmax())
    assert abs(um[i] - 64.63) <= 0.005 * 64.63 and abs(s[i] - 0.850) <= 0.002
    assert abs(vm[j] - 219.36) <= 0.006 * 219.36 and abs(s[j] - 0.0379) <= 0.002
    assert abs(um[i] - 64.83) <= 5e-4 * 64.83 and abs(vm[j] - 220.6) <= 5e-4 * 220.6


def test_cfg4_module_time(cfg4):
    """The cfg4 checks above, oracle assembly included, run in under 60 s on one MI355X."""
    assert time.perf_counter() - _T0["t"] < 60.0
