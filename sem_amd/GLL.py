"""Gauss-Legendre-Lobatto reference element -- drop-in for Solvers/GLL.py.

Same function names, arguments and return shapes as the reference
(Solvers/GLL.py:7-116).  The tables are produced once on the host by
libsemops (sem_amd/csrc/gll_tables.cpp) and are what the device kernels use;
they are tiny ((P+1)^2 doubles), so host generation is the right place for them.
Results are cached per order (the reference recomputes them on every call).
"""
import functools

import numpy as np

from . import _lib


def _arr(n):
    a = np.zeros(n, dtype=np.float64)
    return a, a.ctypes.data_as(_lib._dp)


@functools.lru_cache(maxsize=None)
def _nodes(P: int):
    P = int(P)
    n = P + 1
    x, xp = _arr(n)
    w, wp = _arr(n)
    V, Vp = _arr(n * n)
    _lib.check(_lib.load().sem_gll_nodes(P, xp, wp, Vp))
    for a in (x, w, V):
        a.setflags(write=False)
    return x, w, V.reshape(n, n)


def standard_nodes(P: int):
    """xi[i], w[i], Legendre Vandermonde L_j(xi_i)[i,j]  (GLL.py:7-33)."""
    x, w, V = _nodes(P)
    return x.copy(), w.copy(), V.copy()


@functools.lru_cache(maxsize=None)
def _table(name: str, P: int):
    P = int(P)
    n = P + 1
    a, ap = _arr(n * n)
    _lib.check(getattr(_lib.load(), name)(P, ap))
    a = a.reshape(n, n)
    a.setflags(write=False)
    return a


def standard_mass_matrix(P: int):
    """M_s = diag(w)  (GLL.py:36-42)."""
    return np.diag(_nodes(P)[1])


def standard_differentiation_matrix(P: int):
    """D_s[i,j] = l'_j(xi_i)  (GLL.py:45-59)."""
    return _table("sem_gll_differentiation", P).copy()


def standard_gradient_matrix(P: int):
    """G_s[i,j] = w_i D_s[i,j]  (GLL.py:62-70)."""
    return _table("sem_gll_gradient", P).copy()


def standard_stiffness_matrix(P: int):
    """K_s[i,j] = sum_k w_k D_s[k,i] D_s[k,j]  (GLL.py:73-81)."""
    return _table("sem_gll_stiffness", P).copy()


def standard_product_matrix(P: int):
    """F_s[i,j,k] = w_i delta_ij delta_ik  (GLL.py:84-91)."""
    n = int(P) + 1
    F = np.zeros((n, n, n))
    idx = np.arange(n)
    F[idx, idx, idx] = _nodes(P)[1]
    return F


def standard_convection_matrix(P: int):
    """C_s[i,j,k] = w_i delta_ij D_s[i,k]  (GLL.py:94-102)."""
    n = int(P) + 1
    Cs = np.zeros((n, n, n))
    idx = np.arange(n)
    Cs[idx, idx, :] = _table("sem_gll_gradient", P)
    return Cs


def standard_evaluation_matrix(P: int, xi: np.ndarray):
    """S_s[q,j] = l_j(xi[q])  (GLL.py:105-116)."""
    xi = np.ascontiguousarray(np.asarray(xi, dtype=np.float64).ravel())
    n = int(P) + 1
    S = np.zeros((xi.size, n))
    if xi.size:
        _lib.check(_lib.load().sem_gll_evaluation(int(P), xi.ctypes.data_as(_lib._dp), xi.size,
                                                   S.ctypes.data_as(_lib._dp)))
    return S
