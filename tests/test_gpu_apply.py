"""GPU parity of the fused operator kernel (libsemops via the C ABI) against the
reference's golden vectors and the pinned oracle.

Tolerance: operator applies max|y - y_ref| <= 1e-13 * max|y_ref|
(fp64, different association order than SciPy's CSR SpMV); connectivity, gathers
and the direct-stiffness sum are bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import sem_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-13


def rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


GOLDEN_MESHES = {"P4_4x4": (4, 4, 4, 1.0, 1.0), "P4_3x2": (4, 3, 2, 2.0, 1.0), "P8_8x8": (8, 8, 8, 1.0, 1.0)}


@pytest.mark.parametrize("key", list(GOLDEN_MESHES))
def test_operators_vs_reference_golden(gpu, key):
    from sem_amd import SEM
    P, nex, ney, Lx, Ly = GOLDEN_MESHES[key]
    g = golden("matrices.npz")
    dx, dy = Lx / nex, Ly / ney
    T = g[key + "_T"]
    M = SEM.global_mass_matrix(P, nex, ney, dx, dy)
    K = SEM.global_stiffness_matrix(P, nex, ney, dx, dy)
    Gx, Gy = SEM.global_gradient_matrices(P, nex, ney, dx, dy)
    assert rel(M @ T, g[key + "_MT"]) < TOL
    assert rel(K @ T, g[key + "_KT"]) < TOL
    assert rel(Gx @ T, g[key + "_GxT"]) < TOL
    assert rel(Gy @ T, g[key + "_GyT"]) < TOL
    if key + "_SysT_Pe40" in g:
        Cx, Cy = SEM.global_convection_matrices(P, nex, ney, dx, dy)
        u, v = g[key + "_u"], g[key + "_v"]
        Sys = 40.0 * (SEM.tensordot(Cx, u, (1, 0)) + SEM.tensordot(Cy, v, (1, 0))) + K
        assert rel(Sys @ T, g[key + "_SysT_Pe40"]) < TOL
        # right contraction diag(G_x T) against the reference's own tensor
        import scipy.sparse as sp
        R = sp.csr_matrix((g[key + "_CxT_data"], g[key + "_CxT_indices"], g[key + "_CxT_indptr"]))
        J = SEM.tensordot(Cx, T, (2, 0))
        w = np.random.default_rng(3).uniform(-1, 1, T.size)
        assert rel(J @ w, R @ w) < TOL


def test_tocsr_matches_reference_pattern(gpu):
    from sem_amd import SEM
    g = golden("matrices.npz")
    for key, (P, nex, ney, Lx, Ly) in GOLDEN_MESHES.items():
        dx, dy = Lx / nex, Ly / ney
        ops = {"M": SEM.global_mass_matrix(P, nex, ney, dx, dy), "K": SEM.global_stiffness_matrix(P, nex, ney, dx, dy)}
        ops["Gx"], ops["Gy"] = SEM.global_gradient_matrices(P, nex, ney, dx, dy)
        for nm, op in ops.items():
            A = op.tocsr()
            assert np.array_equal(A.indptr, g[f"{key}_{nm}_indptr"]), (key, nm)
            assert np.array_equal(A.indices, g[f"{key}_{nm}_indices"]), (key, nm)
            assert rel(A.data, g[f"{key}_{nm}_data"]) < 1e-14
            assert rel(op.diagonal(), A.diagonal()) < 1e-14


CASES = [(1, 3, 2), (2, 5, 3), (3, 4, 7), (4, 1, 1), (5, 2, 9), (6, 3, 3), (7, 4, 2), (8, 8, 8), (8, 1, 13),
         (8, 17, 5), (9, 3, 4), (10, 2, 2), (11, 3, 1), (12, 5, 3), (13, 2, 3), (14, 1, 2), (15, 2, 2), (16, 3, 2)]


# VALU two-phase, MFMA (band form, round 5), column kernel, assembled band (+ DPP coefficient variant), and the
# element-block MFMA kernel of rounds 1-4 ("2eb": SEM_MFMA_TILE = 3)
ALGOS = [1, 2, 3, 4, "4dpp", "4imm", "2eb"]
BAND_VARIANTS = {"4dpp": "3", "4imm": "4"}  # SEM_TUNE_BAND_TILE values: DPP-broadcast / immediate coefficients


def _algo(algo, tuning):
    """Select the kernel: an int is sem_apply_desc.algo; a band variant name also sets the band-tile knob."""
    from sem_amd import _lib
    if algo == "2eb":
        tuning(_lib.TUNE_MFMA_TILE, "3")
        return 2
    if isinstance(algo, str):
        tuning(_lib.TUNE_BAND_TILE, BAND_VARIANTS[algo])
        return 4
    return algo


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("P,nex,ney", CASES)
def test_fused_apply_vs_oracle(gpu, P, nex, ney, algo, tuning):
    if algo == "2eb" and P > 15:
        pytest.skip("the element-block MFMA kernel covers P <= 15")
    algo = _algo(algo, tuning)
    from sem_amd.device import get_mesh
    Lx, Ly = 1.3, 0.7
    dx, dy = Lx / nex, Ly / ney
    mesh = get_mesh(P, nex, ney, dx, dy)
    N = mesh.n_local
    r = np.random.default_rng(P * 1000 + nex * 10 + ney)
    x, u, v, a, b = (r.uniform(-1, 1, N) for _ in range(5))
    X, U, V, A, B = (mesh.to_device(t) for t in (x, u, v, a, b))
    ref = {k: O.apply_matrix_free(P, nex, ney, dx, dy, x, **kw) for k, kw in
           {"M": dict(c_mass=1.0), "K": dict(c_stiff=1.0), "Gx": dict(c_gradx=1.0), "Gy": dict(c_grady=1.0)}.items()}
    assert rel(mesh.apply(X, c_mass=1.0, algo=algo), ref["M"]) < TOL
    assert rel(mesh.apply(X, c_stiff=1.0, algo=algo), ref["K"]) < TOL
    assert rel(mesh.apply(X, c_gradx=1.0, algo=algo), ref["Gx"]) < TOL
    assert rel(mesh.apply(X, c_grady=1.0, algo=algo), ref["Gy"]) < TOL
    # everything at once: 0.5 M + K + 40 u.Gx + 40 v.Gy + 3 (a.b + u.v) + 2 y_in
    yin = r.uniform(-1, 1, N)
    Y = mesh.to_device(yin)
    mesh.apply(X, Y, c_mass=0.5, c_stiff=1.0, c_gradx=40.0, cu=U, c_grady=40.0, cv=V, c_extra=3.0, ea=A, eb=B,
               ec=U, ed=V, c_acc=2.0, algo=algo)
    want = 0.5 * ref["M"] + ref["K"] + 40 * u * ref["Gx"] + 40 * v * ref["Gy"] + 3 * (a * b + u * v) + 2 * yin
    assert rel(Y, want) < TOL


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("P,nex,ney", [(4, 4, 4), (8, 6, 5), (12, 3, 4), (8, 40, 33)])
def test_dirichlet_rows(gpu, P, nex, ney, algo, tuning):
    algo = _algo(algo, tuning)
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    mesh = get_mesh(P, nex, ney, 1.0 / nex, 1.0 / ney)
    N, NX, NY = mesh.n_local, mesh.NX, mesh.NY
    r = np.random.default_rng(1)
    x, g = r.uniform(-1, 1, N), r.uniform(-1, 1, N)
    X, G = mesh.to_device(x), mesh.to_device(g)
    base = O.apply_matrix_free(P, nex, ney, 1.0 / nex, 1.0 / ney, x, c_stiff=1.0)
    gx, gy = np.divmod(np.arange(N), NY)
    for sides, sel in ((_lib.SIDE_W | _lib.SIDE_E, (gx == 0) | (gx == NX - 1)),
                       (_lib.SIDE_S, gy == 0), (_lib.SIDE_N | _lib.SIDE_W, (gy == NY - 1) | (gx == 0)),
                       (15, (gx == 0) | (gx == NX - 1) | (gy == 0) | (gy == NY - 1))):
        want = base.copy()
        want[sel] = x[sel] - g[sel]
        y1 = mesh.apply(X, c_stiff=1.0, dir_mode=_lib.DIR_IDENTITY, dir_sides=sides, dir_val=G, algo=algo)
        y2 = mesh.apply(X, c_stiff=1.0, dir_mode=_lib.DIR_IDENTITY,
                        dir_mask=torch.as_tensor(sel.astype(np.uint8), device=mesh.device), dir_val=G, algo=algo)
        assert rel(y1, want) < TOL and torch.equal(y1, y2)
        want[sel] = g[sel]
        y3 = mesh.apply(X, c_stiff=1.0, dir_mode=_lib.DIR_REPLACE, dir_sides=sides, dir_val=G, algo=algo)
        assert rel(y3, want) < TOL
    # an irregular mask (as np.isclose could produce) is honoured row by row
    sel = r.uniform(size=N) < 0.1
    want = base.copy()
    want[sel] = x[sel]
    y = mesh.apply(X, c_stiff=1.0, dir_mode=_lib.DIR_IDENTITY,
                   dir_mask=torch.as_tensor(sel.astype(np.uint8), device=mesh.device), algo=algo)
    assert rel(y, want) < TOL


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("P,nex,ney", [(8, 130, 67), (12, 70, 45), (4, 300, 211)])
def test_large_tiles_vs_oracle(gpu, P, nex, ney, algo, tuning):
    """Meshes big enough for the large-tile / persistent launch configurations."""
    algo = _algo(algo, tuning)
    from sem_amd.device import get_mesh
    dx, dy = 1.0 / nex, 2.0 / ney
    mesh = get_mesh(P, nex, ney, dx, dy)
    N = mesh.n_local
    r = np.random.default_rng(nex + ney)
    x, u, v = (r.uniform(-1, 1, N) for _ in range(3))
    want = (O.apply_matrix_free(P, nex, ney, dx, dy, x, c_stiff=1.0)
            + 40 * O.apply_matrix_free(P, nex, ney, dx, dy, x, c_gradx=1.0, c_grady=1.0, cu=u, cv=v))
    X, U, V = (mesh.to_device(t) for t in (x, u, v))
    y = mesh.apply(X, c_stiff=1.0, c_gradx=40.0, cu=U, c_grady=40.0, cv=V, algo=algo)
    assert rel(y, want) < TOL


@pytest.mark.parametrize("P,nex,ney", [(P, 7, 5) for P in range(1, 17)] + [(8, 64, 64), (8, 3, 70)])
def test_band_variants_bitwise_equal(gpu, P, nex, ney, tuning):
    """The band kernel's coefficient modes (DPP-broadcast lists, fp64 immediates) perform the same operations in
    the same order: results are bitwise identical."""
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    mesh = get_mesh(P, nex, ney, 1.0 / nex, 1.5 / ney)
    r = np.random.default_rng(P)
    X, U, V = (mesh.to_device(r.uniform(-1, 1, mesh.n_local)) for _ in range(3))
    kw = dict(c_mass=0.25, c_stiff=1.0, c_gradx=40.0, cu=U, c_grady=40.0, cv=V, dir_mode=_lib.DIR_IDENTITY,
              dir_sides=_lib.SIDE_W | _lib.SIDE_E, algo=4)
    tuning(_lib.TUNE_BAND_TILE, 0)
    base = mesh.apply(X, **kw)
    for name in ("4dpp", "4imm"):
        tuning(_lib.TUNE_BAND_TILE, BAND_VARIANTS[name])
        assert torch.equal(mesh.apply(X, **kw), base), name


@pytest.mark.parametrize("P,nex,ney,eb,ee", [(8, 64, 64, 0, 64), (8, 40, 13, 10, 30), (4, 9, 7, 2, 9), (12, 5, 3, 0, 5)])
@pytest.mark.parametrize("full", [False, True])
def test_band_kernarg_forms_bitwise_equal(gpu, P, nex, ney, eb, ee, full, tuning):
    """apply_band_kp (prologue fields as preloaded scalar kernel arguments) and apply_band (all
    fields in the struct) run the same body: bitwise-identical results, FULL path included."""
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    mesh = get_mesh(P, nex, ney, 1.0 / nex, 1.5 / ney, eb, ee)
    r = np.random.default_rng(7 * nex + eb)
    N = mesh.n_local
    X, U, V, A, B, Y0, G = (mesh.to_device(r.uniform(-1, 1, N)) for _ in range(7))
    kw = dict(c_mass=0.25, c_stiff=1.0, c_gradx=40.0, cu=U, c_grady=40.0, cv=V, algo=4)
    if full:
        mask = mesh.to_device((r.uniform(0, 1, N) < 0.1).astype(np.uint8), dtype=torch.uint8)
        kw.update(c_extra=3.0, ea=A, eb=B, c_acc=2.0, dir_mode=_lib.DIR_IDENTITY, dir_mask=mask, dir_val=G)
    else:
        kw.update(dir_mode=_lib.DIR_IDENTITY, dir_sides=_lib.SIDE_W | _lib.SIDE_E)
    tuning(_lib.TUNE_BAND_TILE, 0)
    outs = {}
    for kp in (-1, 0):   # -1: struct-only kernel arguments; 0: preloaded prologue arguments
        tuning(_lib.TUNE_BAND_KP, kp)
        outs[kp] = mesh.apply(X, Y0.clone(), **kw)
    assert torch.equal(outs[-1], outs[0])
    # no convection coefficients (cu = cv = None): the preloaded null pointers select the u, v = 1 path
    kw0 = dict(c_stiff=1.0, c_gradx=2.0, c_grady=3.0, algo=4)
    tuning(_lib.TUNE_BAND_KP, -1)
    a0 = mesh.apply(X, **kw0)
    tuning(_lib.TUNE_BAND_KP, 0)
    assert torch.equal(mesh.apply(X, **kw0), a0)


@pytest.mark.parametrize("key", ["P4_4x4", "P4_3x2", "P8_8x8", "P12_5x3"])
def test_gather_and_dss_bit_exact(gpu, key):
    from sem_amd import SEM
    P, nex, ney = {"P4_4x4": (4, 4, 4), "P4_3x2": (4, 3, 2), "P8_8x8": (8, 8, 8), "P12_5x3": (12, 5, 3)}[key]
    g = golden("mesh.npz")
    assert np.array_equal(SEM.scatter(g[key + "_scatter_in"], P, nex, ney), g[key + "_scatter_out"])
    assert np.array_equal(SEM.assemble(g[key + "_assemble4_in"]), g[key + "_assemble4_out"])
    # round trip: DSS of gathered values multiplies each node by its multiplicity
    u = g[key + "_scatter_in"]
    mult = SEM.assemble(np.ones((nex, ney, P + 1, P + 1)))
    assert np.array_equal(SEM.assemble(SEM.scatter(u, P, nex, ney)), u * mult)


def test_cfg2_checksums_full_size(gpu):
    """cfg2 (64x64, P=8, N=263169) against the reference's full-size norms / samples."""
    from sem_amd import SEM
    g = golden("cfg2_checksums.npz")
    N = int(g["N"])
    r = np.random.default_rng(2024)
    T, u, v = r.uniform(-1, 1, N), r.uniform(-1, 1, N), r.uniform(-1, 1, N)
    d = 1.0 / 64
    K = SEM.global_stiffness_matrix(8, 64, 64, d, d)
    Cx, Cy = SEM.global_convection_matrices(8, 64, 64, d, d)
    Sys = 40.0 * (SEM.tensordot(Cx, u, (1, 0)) + SEM.tensordot(Cy, v, (1, 0))) + K
    KT, ST = K @ T, Sys @ T
    assert abs(np.linalg.norm(KT) - float(g["norm_KT"])) < 1e-12 * float(g["norm_KT"])
    assert abs(np.linalg.norm(ST) - float(g["norm_SysT"])) < 1e-12 * float(g["norm_SysT"])
    assert rel(KT[g["sample_idx"]], g["sample_KT"]) < TOL
    assert rel(ST[g["sample_idx"]], g["sample_SysT"]) < TOL
    M = SEM.global_mass_matrix(8, 64, 64, d, d)
    assert rel((M @ T)[g["sample_idx"]], g["sample_MT"]) < TOL


def test_cfg5_checksums_full_size(gpu):
    """cfg5 (128x128, P=12, N=2,362,369) against norms / strided samples of the reference's own
    assembled K, M, G_x, G_y (tests/golden/make_golden.py gen_cfg5), through the fused kernel."""
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    g = golden("cfg5_checksums.npz")
    N = int(g["N"])
    r = np.random.default_rng(2024)
    T, u, v = r.uniform(-1, 1, N), r.uniform(-1, 1, N), r.uniform(-1, 1, N)
    d = 1.0 / 128
    mesh = get_mesh(12, 128, 128, d, d)
    assert mesh.n_local == N
    Td, Ud, Vd = (mesh.to_device(a) for a in (T, u, v))
    KT = mesh.apply(Td, c_stiff=1.0).cpu().numpy()
    ST = mesh.apply(Td, c_stiff=1.0, c_gradx=40.0, cu=Ud, c_grady=40.0, cv=Vd).cpu().numpy()
    MT = mesh.apply(Td, c_mass=1.0).cpu().numpy()
    for y, nk, sk in ((KT, "norm_KT", "sample_KT"), (ST, "norm_SysT", "sample_SysT"), (MT, "norm_MT", "sample_MT")):
        assert abs(np.linalg.norm(y) - float(g[nk])) < 1e-12 * float(g[nk]), nk
        assert rel(y[g["sample_idx"]], g[sk]) < TOL, sk
    # the bench's Dirichlet W/E identity rows on the same operator
    NY = 128 * 12 + 1
    yd = mesh.apply(Td, c_stiff=1.0, c_gradx=40.0, cu=Ud, c_grady=40.0, cv=Vd, dir_mode=_lib.DIR_IDENTITY,
                    dir_sides=_lib.SIDE_W | _lib.SIDE_E).cpu().numpy()
    want = ST.copy()
    want[:NY], want[-NY:] = T[:NY], T[-NY:]
    assert np.array_equal(yd, want)


@pytest.mark.parametrize("P,ne", [(12, 128), (8, 1024)])
def test_full_size_properties(gpu, P, ne):
    """cfg5 (128^2, P=12) and the HBM-regime mesh (1024^2, P=8, N=67M): size-independent
    identities of the assembled operators, plus bitwise determinism."""
    from sem_amd.device import get_mesh
    d = 1.0 / ne
    mesh = get_mesh(P, ne, ne, d, d)
    N = mesh.n_local
    gen = torch.Generator(device=mesh.device).manual_seed(5)
    x = torch.rand(N, dtype=torch.float64, device=mesh.device, generator=gen) * 2 - 1
    z = torch.rand(N, dtype=torch.float64, device=mesh.device, generator=gen) * 2 - 1
    ones = torch.ones(N, dtype=torch.float64, device=mesh.device)
    Kx = mesh.apply(x, c_stiff=1.0)
    scale = Kx.abs().max().item()
    assert mesh.apply(ones, c_stiff=1.0).abs().max().item() < 1e-12 * scale          # constant null space
    Kz = mesh.apply(z, c_stiff=1.0)
    assert abs(torch.dot(z, Kx).item() - torch.dot(x, Kz).item()) < 1e-11 * scale * N ** 0.5  # symmetry
    M1 = mesh.apply(ones, c_mass=1.0)
    assert abs(M1.sum().item() - 1.0) < 1e-12                                         # area of [0,1]^2
    from sem_amd import GLL, SEM
    xs = torch.as_tensor(np.repeat(SEM.global_nodes_1d(P, ne, d), mesh.NY), device=mesh.device)
    # rounding scale of G applied to O(1) data: (d/2) * max w * max_i sum_k |G_s[i,k]| * 2 (shared lines)
    w = GLL.standard_nodes(P)[1]
    gscale = d / 2 * w.max() * 2 * np.abs(GLL.standard_gradient_matrix(P)).sum(axis=1).max()
    assert (mesh.apply(xs, c_gradx=1.0) - M1).abs().max().item() < 1e-14 * gscale     # d(x)/dx = 1
    assert mesh.apply(xs, c_grady=1.0).abs().max().item() < 1e-14 * gscale            # d(x)/dy = 0
    lin = mesh.apply(2.0 * x - 3.0 * z, c_stiff=1.0)
    assert (lin - (2.0 * Kx - 3.0 * Kz)).abs().max().item() < 1e-12 * scale            # linearity
    assert torch.equal(Kx, mesh.apply(x, c_stiff=1.0))                                # deterministic


def test_interpolation_vs_reference(gpu):
    from sem_amd import SEM
    g = golden("cd.npz")
    pe = SEM.element_nodes(4, 4, 4, 0.25, 0.25)
    val = SEM.eval_interpolation(SEM.scatter(g["cfg1_T"], 4, 4, 4), pe, (g["cfg1_plot_x"], g["cfg1_plot_y"]))
    assert np.abs(val - g["cfg1_T_plot"]).max() < 1e-13


def test_bad_arguments_raise(gpu):
    from sem_amd.device import get_mesh
    mesh = get_mesh(4, 3, 3, 0.1, 0.1)
    x = torch.zeros(mesh.n_local, dtype=torch.float64, device=mesh.device)
    with pytest.raises(ValueError):
        mesh.apply(x[:-1], c_stiff=1.0)
    with pytest.raises(ValueError):
        mesh.apply(x, x, c_stiff=1.0)
    with pytest.raises(ValueError):
        mesh.apply(x.float(), c_stiff=1.0)


@pytest.mark.parametrize("P,nex,ney,eb,ee", [(8, 64, 64, 0, 64), (8, 40, 13, 10, 30), (4, 9, 7, 2, 9), (12, 5, 3, 0, 5),
                                             (6, 7, 5, 3, 4), (8, 1024, 8, 0, 1024)])
@pytest.mark.parametrize("full", [False, True])
def test_position_ranges_compose_bitwise(gpu, P, nex, ney, eb, ee, full):
    """sem_apply_desc.pos_*: the interface positions and the interior positions in separate launches
    (the multi-GPU overlap schedule) reproduce one whole-strip launch bitwise, and untouched lines
    keep their previous values."""
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    mesh = get_mesh(P, nex, ney, 1.0 / nex, 1.5 / ney, eb, ee)
    r = np.random.default_rng(nex + 3 * eb)
    N = mesh.n_local
    X, U, V, A, B, Y0, G = (mesh.to_device(r.uniform(-1, 1, N)) for _ in range(7))
    kw = dict(c_mass=0.25, c_stiff=1.0, c_gradx=40.0, cu=U, c_grady=40.0, cv=V)
    if full:
        kw.update(c_extra=3.0, ea=A, eb=B, c_acc=2.0, dir_mode=_lib.DIR_IDENTITY, dir_val=G,
                  dir_sides=_lib.SIDE_W | _lib.SIDE_E | _lib.SIDE_S)
    else:
        kw.update(dir_mode=_lib.DIR_IDENTITY, dir_sides=_lib.SIDE_W | _lib.SIDE_E)
    whole = mesh.apply(X, Y0.clone(), **kw)
    n = ee - eb
    y = Y0.clone()
    mesh.apply(X, y, pos=(0, 1), **kw)
    mesh.apply(X, y, pos=(n, n + 1), **kw)
    if n > 1:
        mesh.apply(X, y, pos=(1, n), **kw)
    assert torch.equal(y, whole)
    # a single position writes only its lines
    y2 = Y0.clone()
    mesh.apply(X, y2, pos=(n, n + 1), **kw)
    NY = mesh.NY
    assert torch.equal(y2[-NY:], whole[-NY:]) and torch.equal(y2[:-NY], Y0[:-NY])
    with pytest.raises(ValueError):
        mesh.apply(X, y2, pos=(0, n + 2), **kw)
    with pytest.raises(RuntimeError):
        mesh.apply(X, y2, pos=(0, 1), algo=_lib.ALGO_MFMA, **kw)
