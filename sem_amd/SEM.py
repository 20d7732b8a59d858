"""Continuous-Galerkin spectral element method -- drop-in for Solvers/SEM.py.

Same function names and arguments as the reference (Solvers/SEM.py:11-273).
Coordinates and connectivity are returned as NumPy arrays exactly as the
reference builds them (bit-exact).  The global operators are returned as
matrix-free device operators (sem_amd.operators.SEMOperator): `A @ x` runs one
fused HIP kernel on the GPU (NumPy in -> NumPy out, device tensor in -> device
tensor out), and `.tocsr()` materialises the reference's CSR for SciPy-only
consumers.  `tensordot` replaces pydata-sparse's for the convection tensors.
"""
import typing

import numpy as np
import torch

from . import GLL, _lib
from .device import get_mesh
from .operators import COO3, ConvectionTensor, SEMOperator, tensordot  # noqa: F401  (re-exported API)


def xi2x(e, xi, dx):
    """Physical coordinate from reference coordinate in element e (SEM.py:11-20)."""
    if np.any(xi > 1) or np.any(xi < -1):
        raise ValueError("xi out of range")
    return dx / 2 * (xi + 1) + dx * e


def x2xi(x, dx) -> typing.Tuple[np.ndarray, np.ndarray]:
    """Element number and reference coordinate of physical coordinate x (SEM.py:23-36)."""
    xi, e = np.modf(np.asarray(x, dtype=np.float64) / dx)
    xi = 2 * xi - 1
    shift = np.isclose(xi, -1) * (e > 0)  # (e, -1) -> (e-1, +1)
    e[shift] -= 1
    xi[shift] = 1
    return e.astype(int), xi


def element_nodes_1d(P, N_ex, dx):
    """x^m_k[m, k] (SEM.py:39-48)."""
    nodes = GLL.standard_nodes(P)[0]
    return np.vstack([xi2x(m, nodes, dx) for m in range(N_ex)])


def global_nodes_1d(P, N_ex, dx):
    """x_p[p]: every element's nodes but its first, with 0 prepended (SEM.py:51-60)."""
    return np.insert(np.ravel(element_nodes_1d(P, N_ex, dx)[:, 1:]), 0, 0)


def element_nodes(P, N_ex, N_ey, dx, dy):
    """[x^mn_kl, y^mn_kl] (SEM.py:63-79)."""
    xe, ye = element_nodes_1d(P, N_ex, dx), element_nodes_1d(P, N_ey, dy)
    pe = np.zeros((2, N_ex, N_ey, P + 1, P + 1))
    pe[0] = xe[:, None, :, None]
    pe[1] = ye[None, :, None, :]
    return pe


def global_nodes(P, N_ex, N_ey, dx, dy):
    """[x_p, y_p], x-major ('ij' meshgrid) (SEM.py:82-94)."""
    x1, y1 = global_nodes_1d(P, N_ex, dx), global_nodes_1d(P, N_ey, dy)
    return np.reshape(np.array(np.meshgrid(x1, y1, indexing="ij")), (2, x1.size * y1.size))


def global_index(P, N_ex, N_ey, m, n, i, j):
    """Global DOF of local node (m, n, i, j) (SEM.py:97-110), vectorised, bit-exact.
    Computed by libsemops (sem_global_index); ValueError on out-of-range indices."""
    arrs = np.broadcast_arrays(*(np.asarray(a, dtype=np.int64) for a in (m, n, i, j)))
    shape = arrs[0].shape
    flat = [np.ascontiguousarray(a.ravel()) for a in arrs]
    out = np.empty(flat[0].size, dtype=np.int64)
    _lib.check(_lib.load().sem_global_index(int(P), int(N_ex), int(N_ey), *(f.ctypes.data_as(_lib._i64p) for f in flat),
                                            out.size, out.ctypes.data_as(_lib._i64p)))
    return out.reshape(shape) if shape else out[0]


def _mesh_for_element_array(A_e):
    nex, ney, P = A_e.shape[0], A_e.shape[1], A_e.shape[2] - 1
    # dx, dy do not enter DSS or gathers; unit widths key a shared handle
    return get_mesh(P, nex, ney, 1.0, 1.0)


def assemble(A_e):
    """Global vector / matrix from an element array (SEM.py:113-146).

    4-D element vectors are summed on the GPU (sem_dss, reference summation
    order, bit-exact).  6-D element matrices are assembled to SciPy CSR and 8-D
    element 3-tensors to a COO3 on the host (setup-time formats; the operators
    themselves never materialise)."""
    if isinstance(A_e, torch.Tensor) and A_e.dim() == 4:
        return _mesh_for_element_array(A_e).dss(A_e)
    A_e = np.asarray(A_e, dtype=np.float64)
    if A_e.ndim == 4:
        return _mesh_for_element_array(A_e).dss(A_e).cpu().numpy()
    if A_e.ndim == 6:
        import scipy.sparse as sp
        nex, ney, P = A_e.shape[0], A_e.shape[1], A_e.shape[2] - 1
        m, n, i, j, k, l = np.nonzero(A_e)
        N = (P * nex + 1) * (P * ney + 1)
        rows = global_index(P, nex, ney, m, n, i, j)
        cols = global_index(P, nex, ney, m, n, k, l)
        return sp.coo_matrix((A_e[m, n, i, j, k, l], (rows, cols)), shape=(N, N)).tocsr()
    if A_e.ndim == 8:  # SEM.py:139-145: a COO 3-tensor (host format; see operators.COO3)
        nex, ney, P = A_e.shape[0], A_e.shape[1], A_e.shape[2] - 1
        m, n, i, j, r, s, k, l = np.nonzero(A_e)
        coords = np.vstack((global_index(P, nex, ney, m, n, i, j), global_index(P, nex, ney, m, n, r, s),
                            global_index(P, nex, ney, m, n, k, l)))
        N = (P * nex + 1) * (P * ney + 1)
        return COO3(coords, A_e[m, n, i, j, r, s, k, l], (N, N, N))
    raise ValueError("assemble supports 4-D (vector), 6-D (matrix) and 8-D (3-tensor) element arrays")


def scatter(u, P, N_ex, N_ey):
    """Element coefficients u^mn_ij from a global vector (SEM.py:149-167), gathered on the GPU."""
    N = (P * N_ex + 1) * (P * N_ey + 1)
    if u.shape[0] != N:
        raise ValueError("Not a valid combination of global coefficients vector, P, N_ex, and N_ey")
    mesh = get_mesh(P, N_ex, N_ey, 1.0, 1.0)
    if isinstance(u, torch.Tensor):
        return mesh.gather_elements(mesh.to_device(u))
    return mesh.gather_elements(mesh.to_device(u)).cpu().numpy()


def global_mass_matrix(P, N_ex, N_ey, dx, dy) -> SEMOperator:
    """M (SEM.py:170-183), matrix-free."""
    return SEMOperator(get_mesh(P, N_ex, N_ey, dx, dy), cM=1.0)


def global_stiffness_matrix(P, N_ex, N_ey, dx, dy) -> SEMOperator:
    """K (SEM.py:186-203), matrix-free."""
    return SEMOperator(get_mesh(P, N_ex, N_ey, dx, dy), cK=1.0)


def global_gradient_matrices(P, N_ex, N_ey, dx, dy) -> typing.Tuple[SEMOperator, SEMOperator]:
    """G_x, G_y (SEM.py:206-223), matrix-free."""
    mesh = get_mesh(P, N_ex, N_ey, dx, dy)
    return SEMOperator(mesh, gx=[(1.0, None)]), SEMOperator(mesh, gy=[(1.0, None)])


def global_convection_matrices(P, N_ex, N_ey, dx, dy) -> typing.Tuple[ConvectionTensor, ConvectionTensor]:
    """C_x, C_y (SEM.py:226-245) as contraction objects: `tensordot(C_x, u, (1, 0))` is the
    operator diag(u) G_x and `tensordot(C_x, T, (2, 0))` the operator diag(G_x T)."""
    mesh = get_mesh(P, N_ex, N_ey, dx, dy)
    return ConvectionTensor(mesh, "x"), ConvectionTensor(mesh, "y")


def eval_interpolation(u_e, points_e, points_plot):
    """u evaluated at the ij-meshgrid points_plot (SEM.py:248-273)."""
    from .interp import eval_interpolation as _ev
    return _ev(u_e, points_e, points_plot)
