"""Batched dense inverses through rocSOLVER's strided-batched LU (the library torch itself links).

torch.linalg.inv on a batch goes through hipblasDgetrfBatched (pointer-array batched LU), which on this
ROCm stack returns wrong blocks for large batches and fails its workspace allocation for 242^2 blocks
beyond 128 of them (tools/inv_repro.py, profiles/r03/inv/).  rocsolver_dgetrf_strided_batched +
rocsolver_dgetri_strided_batched take one contiguous strided batch instead.  The blocks are row-major;
rocSOLVER reads column-major, i.e. it inverts A^T, and (A^T)^-1 stored column-major is A^-1 row-major, so
no transposes are needed.  Library calls only: the factorisation of the element blocks is a plain
batched LU, not a kernel this project writes.
"""
import ctypes as C
import os

import torch

_state = {}


def _libs():
    if "lib" not in _state:
        libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
        try:
            rb = C.CDLL(os.path.join(libdir, "librocblas.so"))
            rs = C.CDLL(os.path.join(libdir, "librocsolver.so"))
        except OSError:
            _state["lib"] = None
            return None
        rb.rocblas_create_handle.argtypes = [C.POINTER(C.c_void_p)]
        rb.rocblas_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        sig = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_int]
        rs.rocsolver_dgetrf_strided_batched.argtypes = [C.c_void_p, C.c_int] + sig[1:]
        rs.rocsolver_dgetri_strided_batched.argtypes = sig
        _state["lib"] = (rb, rs)
    return _state["lib"]


def _handle(dev):
    key = ("h", dev.index)
    if key not in _state:
        rb, _ = _libs()
        h = C.c_void_p()
        if rb.rocblas_create_handle(C.byref(h)) != 0:
            raise RuntimeError("rocblas_create_handle failed")
        _state[key] = h
    return _state[key]


def available():
    return torch.cuda.is_available() and _libs() is not None


def strided_inverse(A):
    """Inverses of a contiguous float64 (nb, n, n) CUDA batch by rocSOLVER strided-batched getrf + getri.
    Returns (X, info) with info the per-block LU status (0: regular; k > 0: exactly singular pivot k)."""
    if not (A.is_cuda and A.dtype == torch.float64 and A.dim() == 3 and A.shape[1] == A.shape[2]):
        raise ValueError("strided_inverse needs a float64 (nb, n, n) CUDA tensor")
    rb, rs = _libs()
    nb, n = A.shape[0], A.shape[1]
    X = A.contiguous().clone()
    ipiv = torch.empty((nb, n), dtype=torch.int32, device=A.device)
    info = torch.empty(nb, dtype=torch.int32, device=A.device)
    h = _handle(A.device)
    rb.rocblas_set_stream(h, C.c_void_p(torch.cuda.current_stream(A.device).cuda_stream))
    p = C.c_void_p
    st = rs.rocsolver_dgetrf_strided_batched(h, n, n, p(X.data_ptr()), n, n * n, p(ipiv.data_ptr()), n,
                                             p(info.data_ptr()), nb)
    if st != 0:
        raise RuntimeError(f"rocsolver_dgetrf_strided_batched: status {st}")
    st = rs.rocsolver_dgetri_strided_batched(h, n, p(X.data_ptr()), n, n * n, p(ipiv.data_ptr()), n,
                                             p(info.data_ptr()), nb)
    if st != 0:
        raise RuntimeError(f"rocsolver_dgetri_strided_batched: status {st}")
    return X, info
