"""Generate golden vectors for the SEM operator layer from the reference itself.

Runs ONLY in the build container, where the read-only reference lives at
/root/reference.  It imports the reference's own `Solvers/GLL.py`, `Solvers/SEM.py`
and the two solver classes, runs them on small seeded cases and writes the
inputs/outputs as .npz fixtures next to this script.  No reference source is
copied; only numbers are written.

Two in-process adapters are needed because this container lacks two pinned
dependencies of the reference (`requirements.txt:1-4`):

* pydata `sparse` 0.12 (absent).  `SEM.py:8` imports it and `SEM.assemble`
  (`SEM.py:139-145`) builds `sparse.COO(coords, data, shape)` for the 8-D
  convection tensors.  The stub below is a plain holder for the (coords, data,
  shape) triplet the reference builds; `tensordot(C, x, (ax, 0))` is restated as
  "sum data * x[coords[ax]] over duplicate remaining coordinates", which is the
  published semantics of pydata-sparse tensordot with a dense vector, followed
  by `.tocsr()` through SciPy's COO->CSR (which sums duplicates).
* SciPy 1.15 removed `lgmres(tol=...)`; the solvers call it with `tol=0`
  (`ConvectionDiffusion_Solver.py:146-148`, `NavierStokes_Solver.py:222-224`).
  The shim forwards `tol` as `rtol` (same meaning in SciPy <1.12).

Usage:  python tests/golden/make_golden.py [--only cfg5|components]
"""
import os
import sys
import types

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- adapters
class _COO:
    """Holder for the (coords, data, shape) triplet `SEM.assemble` builds (SEM.py:145)."""

    def __init__(self, coords, data, shape):
        self.coords = np.asarray(coords).astype(np.int64)
        self.data = np.asarray(data, dtype=np.float64)
        self.shape = tuple(shape)

    def tocsr(self):
        assert len(self.shape) == 2
        return sp.coo_matrix((self.data, (self.coords[0], self.coords[1])), shape=self.shape).tocsr()

    def __mul__(self, s):
        return _COO(self.coords, self.data * s, self.shape)

    __rmul__ = __mul__

    def __add__(self, other):
        return _COO(np.hstack([self.coords, other.coords]), np.hstack([self.data, other.data]), self.shape)


def _tensordot(a, x, axes, return_type=None):
    ax, bx = axes
    assert bx == 0 and np.ndim(x) == 1
    keep = [d for d in range(len(a.shape)) if d != ax]
    data = a.data * np.asarray(x)[a.coords[ax]]
    return _COO(a.coords[keep], data, tuple(a.shape[d] for d in keep))


def install_adapters():
    stub = types.ModuleType("sparse")
    stub.COO = _COO
    stub.tensordot = _tensordot
    sys.modules["sparse"] = stub
    orig = spla.lgmres

    def lgmres(*args, tol=None, **kw):
        if tol is not None:
            kw["rtol"] = tol
        return orig(*args, **kw)

    spla.lgmres = lgmres
    if REF not in sys.path:
        sys.path.insert(0, REF)


def csr_parts(A, prefix):
    A = A.tocsr()
    return {prefix + "_indptr": A.indptr.astype(np.int64), prefix + "_indices": A.indices.astype(np.int64),
            prefix + "_data": A.data.astype(np.float64)}


def rng_fields(N, seed=2024):
    r = np.random.default_rng(seed)
    T = r.uniform(-1, 1, N)
    u = r.uniform(-1, 1, N)
    v = r.uniform(-1, 1, N)
    return T, u, v


# --------------------------------------------------------------------------- fixtures
def gen_gll(GLL):
    d = {}
    for P in range(1, 17):
        x, w, V = GLL.standard_nodes(P)
        d[f"P{P}_x"], d[f"P{P}_w"], d[f"P{P}_V"] = x, w, V
        d[f"P{P}_M"] = GLL.standard_mass_matrix(P)
        d[f"P{P}_D"] = GLL.standard_differentiation_matrix(P)
        d[f"P{P}_G"] = GLL.standard_gradient_matrix(P)
        d[f"P{P}_K"] = GLL.standard_stiffness_matrix(P)
        if P <= 8:
            d[f"P{P}_F"] = GLL.standard_product_matrix(P)
            d[f"P{P}_C"] = GLL.standard_convection_matrix(P)
        xi = np.linspace(-1, 1, 7)
        d[f"P{P}_S"] = GLL.standard_evaluation_matrix(P, xi)
    np.savez_compressed(os.path.join(OUT, "gll.npz"), **d)


MESHES = [(4, 4, 4, 1.0, 1.0), (4, 3, 2, 2.0, 1.0), (8, 8, 8, 1.0, 1.0), (12, 5, 3, 1.0, 1.0)]


def gen_mesh(SEM):
    d = {}
    for (P, nex, ney, Lx, Ly) in MESHES:
        key = f"P{P}_{nex}x{ney}"
        dx, dy = Lx / nex, Ly / ney
        m, n, i, j = np.meshgrid(np.arange(nex), np.arange(ney), np.arange(P + 1), np.arange(P + 1), indexing="ij")
        d[key + "_gidx"] = np.asarray(SEM.global_index(P, nex, ney, m, n, i, j), dtype=np.int64)
        d[key + "_points"] = SEM.global_nodes(P, nex, ney, dx, dy)
        d[key + "_points_e"] = SEM.element_nodes(P, nex, ney, dx, dy)
        d[key + "_dxdy"] = np.array([dx, dy])
        N = (nex * P + 1) * (ney * P + 1)
        r = np.random.default_rng(7)
        u = r.uniform(-1, 1, N)
        d[key + "_scatter_in"] = u
        d[key + "_scatter_out"] = SEM.scatter(u, P, nex, ney)
        a_e = r.uniform(-1, 1, (nex, ney, P + 1, P + 1))
        d[key + "_assemble4_in"] = a_e
        d[key + "_assemble4_out"] = SEM.assemble(a_e)
    np.savez_compressed(os.path.join(OUT, "mesh.npz"), **d)


def gen_matrices(SEM):
    d = {}
    for (P, nex, ney, Lx, Ly) in [(4, 4, 4, 1.0, 1.0), (4, 3, 2, 2.0, 1.0), (8, 8, 8, 1.0, 1.0)]:
        key = f"P{P}_{nex}x{ney}"
        dx, dy = Lx / nex, Ly / ney
        M = SEM.global_mass_matrix(P, nex, ney, dx, dy)
        K = SEM.global_stiffness_matrix(P, nex, ney, dx, dy)
        Gx, Gy = SEM.global_gradient_matrices(P, nex, ney, dx, dy)
        d.update(csr_parts(M, key + "_M"))
        d.update(csr_parts(K, key + "_K"))
        d.update(csr_parts(Gx, key + "_Gx"))
        d.update(csr_parts(Gy, key + "_Gy"))
        N = K.shape[0]
        T, u, v = rng_fields(N)
        d[key + "_T"], d[key + "_u"], d[key + "_v"] = T, u, v
        d[key + "_KT"] = K @ T
        d[key + "_MT"] = M @ T
        d[key + "_GxT"] = Gx @ T
        d[key + "_GyT"] = Gy @ T
        if nex * ney <= 16:
            Cx, Cy = SEM.global_convection_matrices(P, nex, ney, dx, dy)
            uCx = _tensordot(Cx, u, (1, 0)).tocsr()
            vCy = _tensordot(Cy, v, (1, 0)).tocsr()
            CxT = _tensordot(Cx, T, (2, 0)).tocsr()
            CyT = _tensordot(Cy, T, (2, 0)).tocsr()
            d.update(csr_parts(uCx, key + "_uCx"))
            d.update(csr_parts(vCy, key + "_vCy"))
            d.update(csr_parts(CxT, key + "_CxT"))
            d.update(csr_parts(CyT, key + "_CyT"))
            Sys = 40.0 * (uCx + vCy) + K
            d[key + "_SysT_Pe40"] = Sys @ T
    np.savez_compressed(os.path.join(OUT, "matrices.npz"), **d)


def gen_cd(CDS):
    d = {}
    # residual / differential residual through the reference solver class
    for (P, nex, ney, Lx, Ly, bc) in [(4, 4, 4, 1.0, 1.0, dict(T_W=0.5, T_E=-0.5)),
                                      (4, 3, 2, 2.0, 1.0, dict(T_W=0.5, T_E=-0.5, T_S=0.25, T_N=1.0)),
                                      (8, 8, 8, 1.0, 1.0, dict(T_W=0.5, T_E=-0.5))]:
        key = f"P{P}_{nex}x{ney}"
        cd = CDS(Lx, Ly, 40.0, P, nex, ney, **bc)
        T, u, v = rng_fields(cd.N)
        res = cd._get_residuals(T, u, v)
        cd._calc_jacobians(T)
        r = np.random.default_rng(11)
        dT, du, dv = r.uniform(-1, 1, cd.N), r.uniform(-1, 1, cd.N), r.uniform(-1, 1, cd.N)
        dres = cd._get_dresiduals(dT)
        dres_full = cd._get_dresiduals(dT, du, dv)
        d[key + "_bc"] = np.array([bc.get(s, np.nan) for s in ("T_W", "T_E", "T_S", "T_N")])
        d[key + "_LxLy"] = np.array([Lx, Ly])
        d[key + "_T"], d[key + "_u"], d[key + "_v"] = T, u, v
        d[key + "_dT"], d[key + "_du"], d[key + "_dv"] = dT, du, dv
        d[key + "_mask_dir"] = cd._mask_dir
        d[key + "_dirichlet"] = cd._dirichlet
        d[key + "_res"] = res
        d[key + "_dres"] = dres
        d[key + "_dres_full"] = dres_full
    # cfg1: Examples/ConvectionDiffusion_Example.py physics on 4x4, P=4
    cd = CDS(1.0, 1.0, 40.0, 4, 4, 4, T_E=-0.5, T_W=0.5)
    u = cd._get_vector(lambda x, y: y - 0.5)
    v = cd._get_vector(lambda x, y: 0.5 - x)
    Tsol = cd._get_solution(u, v)
    d["cfg1_T"] = Tsol
    d["cfg1_res_after"] = cd._get_residuals(Tsol, u, v)
    xp, yp = np.meshgrid(np.linspace(0, 1, 11), np.linspace(0, 1, 11), indexing="ij")
    d["cfg1_plot_x"], d["cfg1_plot_y"] = xp, yp
    d["cfg1_T_plot"] = cd._get_interpol(Tsol, (xp, yp))
    np.savez_compressed(os.path.join(OUT, "cd.npz"), **d)


def gen_ns(NSS):
    d = {}
    P, nex, ney = 4, 4, 4
    ns = NSS(1.0, 1.0, 100.0, 50.0, P, nex, ney, u_N=1.0, iprint=[])
    r = np.random.default_rng(5)
    u, v, p, T = (r.uniform(-1, 1, ns.N) for _ in range(4))
    ru, rv, rc = ns._get_residuals(u, v, p, T)
    ns._calc_jacobians(u, v)
    du, dv, dp, dT = (r.uniform(-1, 1, ns.N) for _ in range(4))
    dru, drv, drc = ns._get_dresiduals(du, dv, dp, dT)
    for k, a in dict(u=u, v=v, p=p, T=T, du=du, dv=dv, dp=dp, dT=dT, ru=ru, rv=rv, rc=rc,
                     dru=dru, drv=drv, drc=drc, mask_bound=ns._mask_bound, mask_dir_p=ns._mask_dir_p,
                     dir_u=ns._dirichlet_u, dir_v=ns._dirichlet_v).items():
        d["P4_4x4_" + k] = a
    # one lid-driven solve (Re=100) on the same mesh
    ns2 = NSS(1.0, 1.0, 100.0, 0.0, P, nex, ney, u_N=1.0, iprint=[])
    us, vs, ps = ns2._get_solution(np.zeros(ns2.N))
    d["lid_u"], d["lid_v"], d["lid_p"], d["lid_newton_iters"] = us, vs, ps, np.array(ns2._k)
    np.savez_compressed(os.path.join(OUT, "ns.npz"), **d)


def gen_checksums(SEM):
    """Full-size cfg2 (64x64, P=8) checksums: arrays are too big to commit."""
    d = {}
    P, ne = 8, 64
    dx = dy = 1.0 / ne
    K = SEM.global_stiffness_matrix(P, ne, ne, dx, dy)
    M = SEM.global_mass_matrix(P, ne, ne, dx, dy)
    Gx, Gy = SEM.global_gradient_matrices(P, ne, ne, dx, dy)
    N = K.shape[0]
    T, u, v = rng_fields(N)
    KT = K @ T
    GxT, GyT = Gx @ T, Gy @ T
    SysT = KT + 40.0 * (u * GxT + v * GyT)
    d["N"] = np.array(N)
    d["nnz_K"], d["nnz_Gx"], d["nnz_M"] = np.array(K.nnz), np.array(Gx.nnz), np.array(M.nnz)
    d["norm_KT"], d["norm_SysT"] = np.array(np.linalg.norm(KT)), np.array(np.linalg.norm(SysT))
    d["sample_idx"] = np.arange(0, N, 97)
    d["sample_KT"], d["sample_SysT"], d["sample_MT"] = KT[::97], SysT[::97], (M @ T)[::97]
    np.savez_compressed(os.path.join(OUT, "cfg2_checksums.npz"), **d)


def gen_boussinesq(CDS, NSS):
    """Coupled natural convection (OpenMDAO/Boussinesq_SequentialCoupler.py:10-108) with the
    reference's own solver classes, driven by sem_amd.solvers.boussinesq.BoussinesqCoupler (the
    OpenMDAO driver itself is not installed here).  Case "a": equal meshes 4x4 P=4, JNK;
    case "b": CD on 4x4 P=4, NS on 3x3 P=6 (exercises the change_inputs mesh transfers), JNK;
    case "c": same as "a" in NJ mode."""
    sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    d = {}
    cases = {"a": (4, 4, 4, 4, 4, 4, "JNK"), "b": (4, 4, 4, 6, 3, 3, "JNK"), "c": (4, 4, 4, 4, 4, 4, "NJ")}
    for key, (Pc, nxc, nyc, Pn, nxn, nyn, mode) in cases.items():
        Re, Ra, Pr = 1e3, 1e3, 0.71
        cd = CDS(L_x=1.0, L_y=1.0, Pe=Re * Pr, P=Pc, N_ex=nxc, N_ey=nyc, T_W=0.5, T_E=-0.5, mtol=1e-13)
        ns = NSS(L_x=1.0, L_y=1.0, Re=Re, Gr=Ra / Pr, P=Pn, N_ex=nxn, N_ey=nyn, mtol=1e-13, mtol_newton=1e-13,
                 iprint=[])
        c = BoussinesqCoupler(1.0, 1.0, Re, Ra, Pr, Pc, nxc, nyc, Pn, nxn, nyn, mode=mode, cd=cd, ns=ns)
        T, u, v, p = c.solve()
        d[key + "_cfg"] = np.array([Pc, nxc, nyc, Pn, nxn, nyn])
        d[key + "_mode"] = np.array(mode)
        d[key + "_T"], d[key + "_u"], d[key + "_v"], d[key + "_p"] = T, u, v, p
        d[key + "_iters"] = np.array(c.iterations)
        # one coupled residual / Jacobian evaluation at a seeded state
        r = np.random.default_rng(31)
        x = r.uniform(-0.5, 0.5, c.DOF)
        dx = r.uniform(-1, 1, c.DOF)
        d[key + "_x"], d[key + "_dx"] = x, dx
        d[key + "_R"] = c.residuals(x)
        c.linearize(x)
        d[key + "_JR"] = c.jacobian_apply(dx)
    np.savez_compressed(os.path.join(OUT, "bous.npz"), **d)


def gen_components(CDS, NSS):
    """The two OpenMDAO components (OpenMDAO/ConvectionDiffusion_Component.py,
    OpenMDAO/NavierStokes_Component.py) driven method by method, in OpenMDAO's call order, around
    the reference's own solver classes, on mismatched meshes (CD 4x4 P=4, NS 3x3 P=6) so that
    change_inputs interpolates.  OpenMDAO is absent offline: `openmdao.api.ImplicitComponent` is
    the minimal stand-in sem_amd.solvers.components.ImplicitComponent (options.declare,
    add_input/add_output, initialize at construction) -- all the two components touch."""
    sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
    from sem_amd.solvers.components import ImplicitComponent
    pkg, api = types.ModuleType("openmdao"), types.ModuleType("openmdao.api")
    api.ImplicitComponent = ImplicitComponent
    pkg.api = api
    sys.modules["openmdao"], sys.modules["openmdao.api"] = pkg, api
    from OpenMDAO.ConvectionDiffusion_Component import ConvectionDiffusion_Component
    from OpenMDAO.NavierStokes_Component import NavierStokes_Component
    Re, Ra, Pr = 100.0, 1e3, 0.71
    cfg = (4, 4, 4, 6, 3, 3)
    cd = CDS(L_x=1.0, L_y=1.0, Pe=Re * Pr, P=cfg[0], N_ex=cfg[1], N_ey=cfg[2], T_W=0.5, T_E=-0.5, mtol=1e-13)
    ns = NSS(L_x=1.0, L_y=1.0, Re=Re, Gr=Ra / Pr, P=cfg[3], N_ex=cfg[4], N_ey=cfg[5], mtol=1e-13,
             mtol_newton=1e-13, iprint=[])
    d = {"cfg": np.array(cfg), "Re_Ra_Pr": np.array([Re, Ra, Pr])}
    r = np.random.default_rng(47)
    U = lambda n, a=0.5: r.uniform(-a, a, n)  # noqa: E731
    # ---- convection-diffusion component
    c = ConvectionDiffusion_Component(solver_CD=cd, solver_NS=ns)
    c.setup()
    inp = {"u_ns": U(ns.N), "v_ns": U(ns.N)}
    out = {"T_cd": U(cd.N)}
    d["cd_u_ns"], d["cd_v_ns"], d["cd_T"] = inp["u_ns"], inp["v_ns"], out["T_cd"]
    d["cd_change_u"], d["cd_change_v"] = c.change_inputs(inp["u_ns"], inp["v_ns"])
    res = {}
    c.apply_nonlinear(inp, out, res)
    d["cd_res"] = res["T_cd"]
    c.linearize(inp, out, None)
    din, dout, dres = {"u_ns": U(ns.N, 1), "v_ns": U(ns.N, 1)}, {"T_cd": U(cd.N, 1)}, {}
    d["cd_d_u_ns"], d["cd_d_v_ns"], d["cd_dT"] = din["u_ns"], din["v_ns"], dout["T_cd"]
    c.apply_linear(inp, out, din, dout, dres, "fwd")
    d["cd_dres"] = dres["T_cd"]
    c.apply_linear(inp, out, din, {}, dres, "fwd")
    d["cd_dres_no_dT"] = dres["T_cd"]
    rhs = {"T_cd": U(cd.N, 1)}
    dsol = {"T_cd": np.zeros(cd.N)}
    c.solve_linear(dsol, rhs, "fwd")
    d["cd_rhs"], d["cd_solve_linear"] = rhs["T_cd"], dsol["T_cd"]
    out2 = {"T_cd": np.zeros(cd.N)}
    smooth = {"u_ns": ns._get_vector(lambda x, y: 0.2 * (y - 0.5)), "v_ns": ns._get_vector(lambda x, y: 0.2 * (0.5 - x))}
    c.solve_nonlinear(smooth, out2)
    d["cd_smooth_u_ns"], d["cd_smooth_v_ns"] = smooth["u_ns"], smooth["v_ns"]
    d["cd_solve_nonlinear"], d["cd_iter_count"] = out2["T_cd"], np.array(c.iter_count_solve)
    # ---- Navier-Stokes component
    n = NavierStokes_Component(solver_NS=ns, solver_CD=cd)
    n.setup()
    inp = {"T_cd": U(cd.N)}
    out = {k: U(ns.N, 0.2) for k in ("u_ns", "v_ns", "p_ns")}
    d["ns_T_cd"] = inp["T_cd"]
    for k in out:
        d["ns_" + k] = out[k]
    d["ns_change_T"] = n.change_inputs(inp["T_cd"])
    res = {}
    n.apply_nonlinear(inp, out, res)
    for k in res:
        d["ns_res_" + k] = res[k]
    n.linearize(inp, out, None)
    din, dout = {"T_cd": U(cd.N, 1)}, {k: U(ns.N, 1) for k in ("u_ns", "v_ns", "p_ns")}
    d["ns_d_T_cd"] = din["T_cd"]
    for k in dout:
        d["ns_d_" + k] = dout[k]
    dres = {}
    n.apply_linear(inp, out, din, dout, dres, "fwd")
    for k in dres:
        d["ns_dres_" + k] = dres[k]
    dres = {}
    n.apply_linear(inp, out, din, {"u_ns": dout["u_ns"]}, dres, "fwd")
    for k in dres:
        d["ns_dres_partial_" + k] = dres[k]
    # solve_linear: a consistent right-hand side (the Jacobian applied to a known update, T fixed)
    # so the singular pressure mode of the equal-order discretisation does not enter
    dres = {}
    n.apply_linear(inp, out, {"T_cd": np.zeros(cd.N)}, dout, dres, "fwd")
    for k in dres:
        d["ns_rhs_" + k] = dres[k]
    dsol = {k: np.zeros(ns.N) for k in ("u_ns", "v_ns", "p_ns")}
    n.solve_linear(dsol, dres, "fwd")
    for k in dsol:
        d["ns_solve_linear_" + k] = dsol[k]
    # solve_nonlinear: the buoyancy-driven flow of the CD component's temperature
    out2 = {k: np.zeros(ns.N) for k in ("u_ns", "v_ns", "p_ns")}
    n.solve_nonlinear({"T_cd": d["cd_solve_nonlinear"]}, out2)
    for k in out2:
        d["ns_solve_nonlinear_" + k] = out2[k]
    d["ns_iter_count"] = np.array(n.iter_count_solve)
    np.savez_compressed(os.path.join(OUT, "components.npz"), **d)


def gen_cfg5(SEM):
    """Full-size cfg5 (128x128, P=12, N=2,362,369) operator checksums from the reference's own
    assembled matrices (SEM.global_{stiffness,mass,gradient}_matrices, SEM.py:170-223).  The
    reference's 8-D convection tensor is infeasible at this size (~632 GB); the
    convection contraction enters through the identity tensordot(C_x, u, (1,0)) = diag(u) G_x,
    pinned against the reference's own COO triplets at small sizes (matrices.npz)."""
    d = {}
    P, ne = 12, 128
    dx = dy = 1.0 / ne
    K = SEM.global_stiffness_matrix(P, ne, ne, dx, dy)
    M = SEM.global_mass_matrix(P, ne, ne, dx, dy)
    Gx, Gy = SEM.global_gradient_matrices(P, ne, ne, dx, dy)
    N = K.shape[0]
    T, u, v = rng_fields(N)
    KT = K @ T
    SysT = KT + 40.0 * (u * (Gx @ T) + v * (Gy @ T))
    d["N"] = np.array(N)
    d["nnz_K"], d["nnz_Gx"], d["nnz_M"] = np.array(K.nnz), np.array(Gx.nnz), np.array(M.nnz)
    d["norm_KT"], d["norm_SysT"] = np.array(np.linalg.norm(KT)), np.array(np.linalg.norm(SysT))
    d["norm_MT"] = np.array(np.linalg.norm(M @ T))
    d["sample_idx"] = np.arange(0, N, 997)
    d["sample_KT"], d["sample_SysT"], d["sample_MT"] = KT[::997], SysT[::997], (M @ T)[::997]
    np.savez_compressed(os.path.join(OUT, "cfg5_checksums.npz"), **d)


def main():
    install_adapters()
    if "--only" in sys.argv:   # regenerate one fixture: --only cfg5
        from Solvers import SEM
        from Solvers.ConvectionDiffusion_Solver import ConvectionDiffusionSolver
        from Solvers.NavierStokes_Solver import NavierStokesSolver
        which = sys.argv[sys.argv.index("--only") + 1]
        if which == "components":
            gen_components(ConvectionDiffusionSolver, NavierStokesSolver)
        else:
            {"cfg5": gen_cfg5}[which](SEM)
        return
    from Solvers import GLL, SEM
    from Solvers.ConvectionDiffusion_Solver import ConvectionDiffusionSolver
    from Solvers.NavierStokes_Solver import NavierStokesSolver
    gen_gll(GLL)
    gen_mesh(SEM)
    gen_matrices(SEM)
    gen_cd(ConvectionDiffusionSolver)
    gen_ns(NavierStokesSolver)
    gen_checksums(SEM)
    gen_cfg5(SEM)
    gen_boussinesq(ConvectionDiffusionSolver, NavierStokesSolver)
    gen_components(ConvectionDiffusionSolver, NavierStokesSolver)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
