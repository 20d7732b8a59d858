"""Boussinesq coupler counterpart (sem_amd/solvers/boussinesq.py) against the reference solver
classes driven through the same coupling (tests/golden/bous.npz, made by make_golden.py
gen_boussinesq) and against de Vahl Davis' benchmark (the reference example's comment,
Examples/Boussinesq_Sequential_Example.py)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _coupler(g, key):
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    Pc, nxc, nyc, Pn, nxn, nyn = (int(a) for a in g[key + "_cfg"])
    return BoussinesqCoupler(1.0, 1.0, 1e3, 1e3, 0.71, Pc, nxc, nyc, Pn, nxn, nyn, mode=str(g[key + "_mode"]))


@pytest.mark.parametrize("key", ["a", "b", "c"])
def test_coupled_maps(gpu, key):
    """One coupled residual and Jacobian apply at a seeded state: the operator layer's 1e-13 bar
    (case b includes the mesh transfers, whose interpolation is evaluated in fp64)."""
    g = golden("bous.npz")
    c = _coupler(g, key)
    R = c.residuals(g[key + "_x"])
    assert np.abs(R - g[key + "_R"]).max() <= 1e-12 * np.abs(g[key + "_R"]).max()
    c.linearize(g[key + "_x"])
    JR = c.jacobian_apply(g[key + "_dx"])
    assert np.abs(JR - g[key + "_JR"]).max() <= 1e-12 * np.abs(g[key + "_JR"]).max()


@pytest.mark.parametrize("key", ["a", "b", "c"])
def test_coupled_solve(gpu, key):
    """Full coupled solve: same Newton iteration count; fields agree to the nonlinear tolerance
    (||R|| <= 1e-9 sqrt(DOF) on both sides, so the fields differ by ~cond * 1e-9)."""
    g = golden("bous.npz")
    c = _coupler(g, key)
    T, u, v, p = c.solve()
    assert c.iterations == int(g[key + "_iters"])
    for name, a in zip("Tuv", (T, u, v)):
        ref = g[key + "_" + name]
        assert np.abs(a - ref).max() <= 1e-6 * max(np.abs(ref).max(), 1e-3), name
    assert np.linalg.norm(c.residuals(np.concatenate([T, u, v, p]))) <= c.atol_nonlin


def test_de_vahl_davis_ra1e3(gpu):
    """Examples/Boussinesq_Sequential_Example.py at its own settings (P=4, 8x8, Ra=1e3, JNK):
    de Vahl Davis reports u_max*RePr = 3.649, v_max*RePr = 3.697 for Ra = 1e3."""
    from sem_amd.solvers.boussinesq import run
    x, y = np.meshgrid(np.linspace(0, 1, 101), np.linspace(0, 1, 101), indexing="ij")
    T, u, v = run((x, y), 1.0, 1.0, 1e3, 1e3, 0.71, 4, 8, 8, 4, 8, 8, mode="JNK")
    assert abs(u.max() * 710 - 3.649) < 0.01 * 3.649
    assert abs(v.max() * 710 - 3.697) < 0.01 * 3.697
    assert np.abs(T).max() <= 0.5 + 1e-9


def test_de_vahl_davis_ra1e4_midlines(gpu):
    """cfg4's physics on a 16^2, P=8 mesh: the JNK coupler from rest through Ra = 1e3 to Ra = 1e4
    (continuation through the coupler's initial guess, as tools/bous_solve.py runs cfg4), then the
    de Vahl Davis (1983) midline maxima: u_max*RePr = 16.178 at y = 0.823 on x = 1/2 and
    v_max*RePr = 19.617 at x = 0.119 on y = 1/2."""
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    x = None
    for Ra in (1e3, 1e4):
        c = BoussinesqCoupler(1.0, 1.0, 1e3, Ra, 0.71, 8, 16, 16, 8, 16, 16, mode="JNK")
        x = np.concatenate(c.solve(x))
    N = c.Nns
    u, v = x[c.Ncd:c.Ncd + N], x[c.Ncd + N:c.Ncd + 2 * N]
    s = np.linspace(0.0, 1.0, 1001)
    um = np.asarray(c.ns._get_interpol(u, np.meshgrid([0.5], s, indexing="ij")))[0] * 710.0
    vm = np.asarray(c.ns._get_interpol(v, np.meshgrid(s, [0.5], indexing="ij")))[:, 0] * 710.0
    assert abs(um.max() - 16.178) < 0.005 * 16.178 and abs(s[um.argmax()] - 0.823) <= 0.004
    assert abs(vm.max() - 19.617) < 0.005 * 19.617 and abs(s[vm.argmax()] - 0.119) <= 0.004
