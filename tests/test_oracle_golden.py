"""Pin the oracle (oracle/sem_oracle.py) against golden vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from conftest import golden
from oracle import sem_oracle as O

MESHES = {"P4_4x4": (4, 4, 4, 1.0, 1.0), "P4_3x2": (4, 3, 2, 2.0, 1.0), "P8_8x8": (8, 8, 8, 1.0, 1.0),
          "P12_5x3": (12, 5, 3, 1.0, 1.0)}


def rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("P", range(1, 17))
def test_gll_tables(P):
    g = golden("gll.npz")
    x, w, V = O.gll_nodes(P)
    assert np.array_equal(x, g[f"P{P}_x"]) and np.array_equal(w, g[f"P{P}_w"]) and np.array_equal(V, g[f"P{P}_V"])
    assert np.array_equal(O.gll_D(P), g[f"P{P}_D"])
    assert np.allclose(O.gll_G(P), g[f"P{P}_G"], rtol=0, atol=1e-14 * P * P)
    assert np.allclose(O.gll_K(P), g[f"P{P}_K"], rtol=0, atol=1e-15 * P ** 3)
    assert np.allclose(O.gll_eval(P, np.linspace(-1, 1, 7)), g[f"P{P}_S"], rtol=0, atol=1e-13)


@pytest.mark.parametrize("key", list(MESHES))
def test_mesh_connectivity_bit_exact(key):
    P, nex, ney, Lx, Ly = MESHES[key]
    g = golden("mesh.npz")
    dx, dy = Lx / nex, Ly / ney
    assert np.array_equal(O._gidx_table(P, nex, ney), g[key + "_gidx"])
    assert np.array_equal(O.global_nodes(P, nex, ney, dx, dy), g[key + "_points"])
    assert np.array_equal(O.element_nodes(P, nex, ney, dx, dy), g[key + "_points_e"])
    assert np.array_equal(O.scatter(g[key + "_scatter_in"], P, nex, ney), g[key + "_scatter_out"])
    assert np.array_equal(O.assemble(g[key + "_assemble4_in"]), g[key + "_assemble4_out"])


@pytest.mark.parametrize("key", ["P4_4x4", "P4_3x2", "P8_8x8"])
def test_assembled_matrices(key):
    P, nex, ney, Lx, Ly = MESHES[key]
    g = golden("matrices.npz")
    dx, dy = Lx / nex, Ly / ney
    M = O.global_mass_matrix(P, nex, ney, dx, dy)
    K = O.global_stiffness_matrix(P, nex, ney, dx, dy)
    Gx, Gy = O.global_gradient_matrices(P, nex, ney, dx, dy)
    for nm, A in (("M", M), ("K", K), ("Gx", Gx), ("Gy", Gy)):
        assert np.array_equal(A.indptr, g[f"{key}_{nm}_indptr"]), nm
        assert np.array_equal(A.indices, g[f"{key}_{nm}_indices"]), nm
        assert rel(A.data, g[f"{key}_{nm}_data"]) < 1e-14, nm
    T, u, v = g[key + "_T"], g[key + "_u"], g[key + "_v"]
    assert rel(K @ T, g[key + "_KT"]) < 1e-13
    assert rel(O.apply_matrix_free(P, nex, ney, dx, dy, T, c_stiff=1.0), g[key + "_KT"]) < 1e-13
    assert rel(O.apply_matrix_free(P, nex, ney, dx, dy, T, c_mass=1.0), g[key + "_MT"]) < 1e-13
    assert rel(O.apply_matrix_free(P, nex, ney, dx, dy, T, c_gradx=1.0), g[key + "_GxT"]) < 1e-13
    assert rel(O.apply_matrix_free(P, nex, ney, dx, dy, T, c_grady=1.0), g[key + "_GyT"]) < 1e-13
    if key + "_uCx_data" in g:
        # the convection identities the oracle relies on, against the reference's own COO triplets
        for nm, A in (("uCx", O.conv_left(Gx, u)), ("vCy", O.conv_left(Gy, v)),
                      ("CxT", O.conv_right(Gx, T)), ("CyT", O.conv_right(Gy, T))):
            import scipy.sparse as sp
            R = sp.csr_matrix((g[f"{key}_{nm}_data"], g[f"{key}_{nm}_indices"], g[f"{key}_{nm}_indptr"]),
                              shape=A.shape)
            assert abs(A - R).max() <= 1e-14 * abs(R).max(), nm
        Sys = 40.0 * (O.conv_left(Gx, u) + O.conv_left(Gy, v)) + K
        assert rel(Sys @ T, g[key + "_SysT_Pe40"]) < 1e-13


@pytest.mark.parametrize("key", ["P4_4x4", "P4_3x2", "P8_8x8"])
def test_cd_operator_applies(key):
    g = golden("cd.npz")
    P, nex, ney = MESHES[key][:3]
    Lx, Ly = g[key + "_LxLy"]
    bc = dict(zip(("T_W", "T_E", "T_S", "T_N"), g[key + "_bc"]))
    bc = {k: float(v) for k, v in bc.items() if not np.isnan(v)}
    cd = O.CDOracle(Lx, Ly, 40.0, P, nex, ney, **bc)
    assert np.array_equal(cd.mask, g[key + "_mask_dir"])
    assert np.array_equal(np.isnan(cd.dirichlet), np.isnan(g[key + "_dirichlet"]))
    res = cd.residuals(g[key + "_T"], g[key + "_u"], g[key + "_v"])
    assert rel(res, g[key + "_res"]) < 1e-13
    cd.calc_jacobians(g[key + "_T"])
    assert rel(cd.dresiduals(g[key + "_dT"]), g[key + "_dres"]) < 1e-13
    assert rel(cd.dresiduals(g[key + "_dT"], g[key + "_du"], g[key + "_dv"]), g[key + "_dres_full"]) < 1e-13


def test_cd_cfg1_solution():
    g = golden("cd.npz")
    cd = O.CDOracle(1.0, 1.0, 40.0, 4, 4, 4, T_E=-0.5, T_W=0.5)
    x, y = cd.points
    T = cd.solution(y - 0.5, 0.5 - x)
    assert np.abs(T - g["cfg1_T"]).max() < 1e-6
    pe = O.element_nodes(4, 4, 4, 0.25, 0.25)
    val = O.eval_interpolation(O.scatter(g["cfg1_T"], 4, 4, 4), pe, (g["cfg1_plot_x"], g["cfg1_plot_y"]))
    assert np.abs(val - g["cfg1_T_plot"]).max() < 1e-13


def test_ns_operator_applies():
    g = golden("ns.npz")
    k = "P4_4x4_"
    ns = O.NSOracle(1.0, 1.0, 100.0, 50.0, 4, 4, 4, u_N=1.0)
    assert np.array_equal(ns.mask_bound, g[k + "mask_bound"]) and np.array_equal(ns.mask_p, g[k + "mask_dir_p"])
    ru, rv, rc = ns.residuals(g[k + "u"], g[k + "v"], g[k + "p"], g[k + "T"])
    assert rel(ru, g[k + "ru"]) < 1e-13 and rel(rv, g[k + "rv"]) < 1e-13 and rel(rc, g[k + "rc"]) < 1e-13
    ns.calc_jacobians(g[k + "u"], g[k + "v"])
    du, dv, dp = ns.dresiduals(g[k + "du"], g[k + "dv"], g[k + "dp"], g[k + "dT"])
    assert rel(du, g[k + "dru"]) < 1e-13 and rel(dv, g[k + "drv"]) < 1e-13 and rel(dp, g[k + "drc"]) < 1e-13


def test_cfg2_checksums():
    """Full-size cfg2 (64x64, P=8): the oracle's assembled K reproduces the reference's
    nnz, norms and sampled entries."""
    g = golden("cfg2_checksums.npz")
    P, ne = 8, 64
    d = 1.0 / ne
    N = int(g["N"])
    r = np.random.default_rng(2024)
    T, u, v = r.uniform(-1, 1, N), r.uniform(-1, 1, N), r.uniform(-1, 1, N)
    y = O.apply_matrix_free(P, ne, ne, d, d, T, c_stiff=1.0)
    assert abs(np.linalg.norm(y) - float(g["norm_KT"])) < 1e-12 * float(g["norm_KT"])
    assert rel(y[g["sample_idx"]], g["sample_KT"]) < 1e-13
    s = y + 40.0 * O.apply_matrix_free(P, ne, ne, d, d, T, c_gradx=1.0, c_grady=1.0, cu=u, cv=v)
    assert rel(s[g["sample_idx"]], g["sample_SysT"]) < 1e-13
