"""CPU tests of the product's host side: the C-ABI library loads and exports every
symbol of include/sem_ops.h, host tables / connectivity are bit-exact with the
reference's golden vectors, and errors map to the reference's exception types.
No device compute here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden
from sem_amd import GLL, SEM, _lib

MESHES = {"P4_4x4": (4, 4, 4, 1.0, 1.0), "P4_3x2": (4, 3, 2, 2.0, 1.0), "P8_8x8": (8, 8, 8, 1.0, 1.0),
          "P12_5x3": (12, 5, 3, 1.0, 1.0)}


def header_functions():
    text = open(os.path.join(ROOT, "include", "sem_ops.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sem_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    declared = header_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(_lib.exported_symbols()) == declared
    assert lib.sem_abi_version() == _lib.ABI_VERSION == 15
    assert lib.sem_max_order() == 16


def test_library_is_in_tree_and_has_gfx950_code():
    assert os.path.commonpath([_lib.LIB_PATH, ROOT]) == ROOT
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("P", range(1, 17))
def test_gll_tables_bit_exact(P):
    g = golden("gll.npz")
    x, w, V = GLL.standard_nodes(P)
    assert np.array_equal(x, g[f"P{P}_x"]) and np.array_equal(w, g[f"P{P}_w"]) and np.array_equal(V, g[f"P{P}_V"])
    assert np.array_equal(GLL.standard_mass_matrix(P), g[f"P{P}_M"])
    assert np.array_equal(GLL.standard_differentiation_matrix(P), g[f"P{P}_D"])
    assert np.array_equal(GLL.standard_gradient_matrix(P), g[f"P{P}_G"])
    assert np.array_equal(GLL.standard_stiffness_matrix(P), g[f"P{P}_K"])
    assert np.array_equal(GLL.standard_evaluation_matrix(P, np.linspace(-1, 1, 7)), g[f"P{P}_S"])
    if P <= 8:
        assert np.array_equal(GLL.standard_product_matrix(P), g[f"P{P}_F"])
        assert np.array_equal(GLL.standard_convection_matrix(P), g[f"P{P}_C"])


def test_gll_properties():
    for P in (2, 5, 8, 12, 16):
        x, w, _ = GLL.standard_nodes(P)
        D = GLL.standard_differentiation_matrix(P)
        K = GLL.standard_stiffness_matrix(P)
        assert abs(w.sum() - 2.0) < 1e-13
        assert np.abs(D @ np.ones(P + 1)).max() < 1e-10 * P * P          # derivative of a constant
        assert np.abs(D @ x - 1.0).max() < 1e-10 * P * P                  # derivative of xi
        assert np.abs(K - K.T).max() < 1e-12 * np.abs(K).max()            # symmetric
        assert np.abs(K @ np.ones(P + 1)).max() < 1e-10 * np.abs(K).max() # constant null space
        assert np.linalg.eigvalsh(K).min() > -1e-10 * np.abs(K).max()     # PSD


@pytest.mark.parametrize("key", list(MESHES))
def test_connectivity_bit_exact(key):
    P, nex, ney, Lx, Ly = MESHES[key]
    g = golden("mesh.npz")
    dx, dy = Lx / nex, Ly / ney
    m, n, i, j = np.meshgrid(np.arange(nex), np.arange(ney), np.arange(P + 1), np.arange(P + 1), indexing="ij")
    assert np.array_equal(SEM.global_index(P, nex, ney, m, n, i, j), g[key + "_gidx"])
    assert np.array_equal(SEM.global_nodes(P, nex, ney, dx, dy), g[key + "_points"])
    assert np.array_equal(SEM.element_nodes(P, nex, ney, dx, dy), g[key + "_points_e"])
    assert SEM.global_index(P, nex, ney, 0, 0, 1, 2) == 2 + (ney * P + 1)


def test_global_index_errors_like_reference():
    with pytest.raises(ValueError):
        SEM.global_index(4, 3, 2, 3, 0, 0, 0)   # m >= N_ex
    with pytest.raises(ValueError):
        SEM.global_index(4, 3, 2, 0, 0, 5, 0)   # i > P
    with pytest.raises(ValueError):
        SEM.xi2x(0, np.array([1.5]), 0.1)


def test_x2xi_shifts_shared_nodes_left():
    e, xi = SEM.x2xi(np.array([0.0, 0.25, 0.3, 1.0]), 0.25)
    assert list(e) == [0, 0, 1, 3]
    assert xi[0] == -1 and xi[1] == 1 and xi[3] == 1


def test_abi_error_paths_without_gpu():
    lib = _lib.load()
    h = C.c_void_p()
    assert lib.sem_create(0, 4, 4, 0.1, 0.1, 0, 4, 0, C.byref(h)) == _lib.SEM_EUNSUPPORTED
    assert lib.sem_create(4, 4, 4, -0.1, 0.1, 0, 4, 0, C.byref(h)) == _lib.SEM_EINVAL
    assert lib.sem_create(4, 4, 4, 0.1, 0.1, 2, 2, 0, C.byref(h)) == _lib.SEM_EINVAL
    assert b"range" in lib.sem_last_error()
    assert lib.sem_apply(None, None, None, None, None) == _lib.SEM_EINVAL
    with pytest.raises(ValueError):
        _lib.check(_lib.SEM_EINVAL)


def test_release_build_has_no_diagnostic_path():
    """no environment variable can change results.  The shipped library is built with
    SEM_DIAGNOSTICS=0 (the SEM_DIAG ablation bits and stamp buffer are compiled out) and its build
    id matches the in-tree sources."""
    from sem_amd.build import source_hash
    lib = _lib.load()
    bid = lib.sem_build_id().decode()
    assert bid == source_hash() and not bid.endswith("+diag")
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"SEM_DIAG" not in blob


def test_tuning_knobs_set_and_get():
    lib = _lib.load()
    v = C.c_int()
    _lib.check(lib.sem_get_tuning(_lib.TUNE_BAND_TILE, C.byref(v)))
    old = v.value
    _lib.check(lib.sem_set_tuning(_lib.TUNE_BAND_TILE, 3))
    _lib.check(lib.sem_get_tuning(_lib.TUNE_BAND_TILE, C.byref(v)))
    assert v.value == 3
    _lib.check(lib.sem_set_tuning(_lib.TUNE_BAND_TILE, old))
    assert lib.sem_set_tuning(99, 1) == _lib.SEM_EINVAL
    for knob in _lib.TUNE_RETIRED:           # round 6: the knobs whose A/B lost are refused
        assert lib.sem_set_tuning(knob, 1) == _lib.SEM_EINVAL
    assert lib.sem_get_tuning(-1, C.byref(v)) == _lib.SEM_EINVAL


def test_loader_refuses_library_from_other_sources(monkeypatch):
    """A library whose build id differs from the in-tree source hash is refused (a stale .so
    would make the GPU tests validate old kernels)."""
    from sem_amd import build
    lib = _lib.load()
    monkeypatch.setattr(build, "source_hash", lambda: "0" * 16)
    with pytest.raises(RuntimeError, match="not built from the sources"):
        _lib._check_build_id(lib)


@pytest.mark.parametrize("key", ["P4_4x4", "P4_3x2"])
def test_assemble_8d_convection_tensor_matches_reference(key):
    """SEM.assemble of an 8-D element array returns the reference's COO 3-tensor (SEM.py:139-145);
    its contractions tensordot(C, u, (1,0)) / tensordot(C, T, (2,0)) reproduce the reference's own
    CSR results (tests/golden/matrices.npz, made from the reference's COO triplets) bit for bit.
    The element tensors are built as SEM.global_convection_matrices does (SEM.py:240-244)."""
    P, nex, ney, Lx, Ly = MESHES[key]
    dx, dy = Lx / nex, Ly / ney
    g = golden("matrices.npz")
    F_s, C_s = GLL.standard_product_matrix(P), GLL.standard_convection_matrix(P)
    F_ex = np.multiply.outer(np.full(nex, dx / 2), F_s)
    F_ey = np.multiply.outer(np.full(ney, dy / 2), F_s)
    C_x_e = np.einsum('m,irk,njsl->mnijrskl', np.ones(nex), C_s, F_ey, optimize=True)
    C_y_e = np.einsum('mirk,n,jsl->mnijrskl', F_ex, np.ones(ney), C_s, optimize=True)
    Cx, Cy = SEM.assemble(C_x_e), SEM.assemble(C_y_e)
    N = (P * nex + 1) * (P * ney + 1)
    assert Cx.shape == (N, N, N)
    for nm, C, vec, ax in (("uCx", Cx, g[key + "_u"], 1), ("vCy", Cy, g[key + "_v"], 1),
                           ("CxT", Cx, g[key + "_T"], 2), ("CyT", Cy, g[key + "_T"], 2)):
        A = SEM.tensordot(C, vec, (ax, 0)).tocsr()
        assert np.array_equal(A.indptr, g[f"{key}_{nm}_indptr"]), nm
        assert np.array_equal(A.indices, g[f"{key}_{nm}_indices"]), nm
        assert np.array_equal(A.data, g[f"{key}_{nm}_data"]), nm
