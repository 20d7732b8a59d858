"""OpenMDAO component counterparts (sem_amd/solvers/components.py) against the reference's own
components (OpenMDAO/ConvectionDiffusion_Component.py, OpenMDAO/NavierStokes_Component.py) driven
method by method in OpenMDAO's call order around the reference solver classes, on mismatched
meshes so change_inputs interpolates (tests/golden/components.npz, make_golden.py gen_components).

The same driver runs twice: on the CPU around the oracle's solver doubles (tests/oracle_solvers.py:
the component logic -- variables, call order, change_inputs, absent-derivative handling, errors,
iteration counts), and with @pytest.mark.gpu around the device solver counterparts (every apply a
HIP launch)."""
import numpy as np
import pytest

from conftest import golden

OUT_NS = ("u_ns", "v_ns", "p_ns")


def _solvers(g, device):
    Re, Ra, Pr = (float(a) for a in g["Re_Ra_Pr"])
    Pc, nxc, nyc, Pn, nxn, nyn = (int(a) for a in g["cfg"])
    if device:
        from sem_amd.solvers import ConvectionDiffusionSolver, NavierStokesSolver
        cd = ConvectionDiffusionSolver(1.0, 1.0, Re * Pr, Pc, nxc, nyc, T_W=0.5, T_E=-0.5, mtol=1e-13)
        ns = NavierStokesSolver(1.0, 1.0, Re, Ra / Pr, Pn, nxn, nyn, mtol=1e-13, mtol_newton=1e-13, iprint=[])
    else:
        from oracle_solvers import OracleCD, OracleNS
        cd = OracleCD(1.0, 1.0, Re * Pr, Pc, nxc, nyc, T_W=0.5, T_E=-0.5, mtol=1e-13)
        ns = OracleNS(1.0, 1.0, Re, Ra / Pr, Pn, nxn, nyn, mtol=1e-13, mtol_newton=1e-13)
    return cd, ns


def _close(a, ref, rel):
    a, ref = np.asarray(a), np.asarray(ref)
    assert a.shape == ref.shape
    return np.abs(a - ref).max() <= rel * max(np.abs(ref).max(), 1e-3)


def _check_cd(g, cd, ns):
    from sem_amd.solvers.components import ConvectionDiffusion_Component
    c = ConvectionDiffusion_Component(solver_CD=cd, solver_NS=ns)
    c.setup()
    assert c.variables["T_cd"][0] == "output" and c.variables["T_cd"][1].shape == (cd.N,)
    assert c.variables["u_ns"][0] == "input" and c.variables["v_ns"][1].shape == (ns.N,)
    inp = {"u_ns": g["cd_u_ns"], "v_ns": g["cd_v_ns"]}
    out = {"T_cd": g["cd_T"]}
    cu, cv = c.change_inputs(inp["u_ns"], inp["v_ns"])
    assert _close(cu, g["cd_change_u"], 1e-13) and _close(cv, g["cd_change_v"], 1e-13)
    res = {}
    c.apply_nonlinear(inp, out, res)
    assert _close(res["T_cd"], g["cd_res"], 1e-12)
    c.linearize(inp, out, None)
    din, dout, dres = {"u_ns": g["cd_d_u_ns"], "v_ns": g["cd_d_v_ns"]}, {"T_cd": g["cd_dT"]}, {}
    c.apply_linear(inp, out, din, dout, dres, "fwd")
    assert _close(dres["T_cd"], g["cd_dres"], 1e-12)
    c.apply_linear(inp, out, din, {}, dres, "fwd")          # d_outputs without T_cd: dT = 0
    assert _close(dres["T_cd"], g["cd_dres_no_dT"], 1e-12)
    with pytest.raises(ValueError, match="only forward mode"):
        c.apply_linear(inp, out, din, dout, dres, "rev")
    dsol = {"T_cd": np.zeros(cd.N)}
    c.solve_linear(dsol, {"T_cd": g["cd_rhs"]}, "fwd")
    assert c.iter_count_solve == 1
    assert _close(dsol["T_cd"], g["cd_solve_linear"], 1e-8)
    with pytest.raises(ValueError, match="only forward mode"):
        c.solve_linear(dsol, {"T_cd": g["cd_rhs"]}, "rev")
    out2 = {"T_cd": np.zeros(cd.N)}
    c.solve_nonlinear({"u_ns": g["cd_smooth_u_ns"], "v_ns": g["cd_smooth_v_ns"]}, out2)
    assert c.iter_count_solve == int(g["cd_iter_count"])
    assert _close(out2["T_cd"], g["cd_solve_nonlinear"], 1e-8)


def _check_ns(g, cd, ns):
    from sem_amd.solvers.components import NavierStokes_Component
    n = NavierStokes_Component(solver_NS=ns, solver_CD=cd)
    n.setup()
    assert [n.variables[k][0] for k in ("T_cd",) + OUT_NS] == ["input", "output", "output", "output"]
    inp = {"T_cd": g["ns_T_cd"]}
    out = {k: g["ns_" + k] for k in OUT_NS}
    assert _close(n.change_inputs(inp["T_cd"]), g["ns_change_T"], 1e-13)
    res = {}
    n.apply_nonlinear(inp, out, res)
    for k in OUT_NS:
        assert _close(res[k], g["ns_res_" + k], 1e-12), k
    n.linearize(inp, out, None)
    din, dout = {"T_cd": g["ns_d_T_cd"]}, {k: g["ns_d_" + k] for k in OUT_NS}
    dres = {}
    n.apply_linear(inp, out, din, dout, dres, "fwd")
    for k in OUT_NS:
        assert _close(dres[k], g["ns_dres_" + k], 1e-12), k
    dres = {}
    n.apply_linear(inp, out, din, {"u_ns": dout["u_ns"]}, dres, "fwd")   # v_ns, p_ns absent: zero
    for k in OUT_NS:
        assert _close(dres[k], g["ns_dres_partial_" + k], 1e-12), k
    with pytest.raises(ValueError, match="only forward mode"):
        n.apply_linear(inp, out, din, dout, dres, "rev")
    # solve_linear on a consistent right-hand side: velocities agree; the pressure is unique only up
    # to the equal-order discretisation's spurious modes, so it is checked through the residual
    rhs = {k: g["ns_rhs_" + k] for k in OUT_NS}
    dsol = {k: np.zeros(ns.N) for k in OUT_NS}
    n.solve_linear(dsol, rhs, "fwd")
    assert n.iter_count_solve == 1
    for k in ("u_ns", "v_ns"):
        assert _close(dsol[k], g["ns_solve_linear_" + k], 1e-6), k
    back = {}
    n.apply_linear(inp, out, {"T_cd": np.zeros(cd.N)}, dsol, back, "fwd")
    scale = max(np.abs(rhs[k]).max() for k in OUT_NS)
    for k in OUT_NS:
        assert np.abs(back[k] - rhs[k]).max() <= 1e-7 * scale, k
    # solve_nonlinear: the inner Newton iteration, counted by its number of updates
    out2 = {k: np.zeros(ns.N) for k in OUT_NS}
    n.solve_nonlinear({"T_cd": g["cd_solve_nonlinear"]}, out2)
    assert n.iter_count_solve == int(g["ns_iter_count"])   # 1 (solve_linear) + Newton updates
    for k in ("u_ns", "v_ns"):
        assert _close(out2[k], g["ns_solve_nonlinear_" + k], 1e-6), k
    r = {}
    n.apply_nonlinear({"T_cd": g["cd_solve_nonlinear"]}, out2, r)
    assert np.sqrt(sum(np.sum(np.square(r[k])) for k in OUT_NS)) <= 1e-13 * np.sqrt(3 * ns.N)


def test_components_oracle_cd():
    g = golden("components.npz")
    _check_cd(g, *_solvers(g, device=False))


def test_components_oracle_ns():
    g = golden("components.npz")
    _check_ns(g, *_solvers(g, device=False))


def test_component_options():
    """om.ImplicitComponent behaviour the components rely on: declared options only, required
    options raise until set, variables recorded at setup."""
    from sem_amd.solvers.components import ConvectionDiffusion_Component
    c = ConvectionDiffusion_Component()
    with pytest.raises(RuntimeError, match="required"):
        c.setup()
    with pytest.raises(KeyError):
        c.options["solver_XY"] = None
    assert "solver_CD" in c.options and "solver_NS" in c.options


@pytest.mark.gpu
def test_components_device_cd(gpu):
    g = golden("components.npz")
    _check_cd(g, *_solvers(g, device=True))


@pytest.mark.gpu
def test_components_device_ns(gpu):
    g = golden("components.npz")
    _check_ns(g, *_solvers(g, device=True))
