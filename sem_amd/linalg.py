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
    """One rocBLAS handle per device, created with that device current (rocblas_create_handle binds the
    handle to the current device)."""
    key = ("h", dev.index)
    if key not in _state:
        rb, _ = _libs()
        h = C.c_void_p()
        with torch.cuda.device(dev):
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
    with torch.cuda.device(A.device):
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


def _split(n):
    """Leading block size of a 2 x 2 split: half of n, rounded up to a multiple of 64 (GEMM tiles)."""
    h = (n // 2 + 63) // 64 * 64
    return h if h < n else n // 2


def block_inverse(A, base=64, out=None):
    """Inverse of one square float64 matrix by 2 x 2 block recursion, all but the leaves in GEMMs:
        A = [[A11, A12], [A21, A22]],  X11 = A11^-1,  T = X11 A12,  U = A21 X11,
        S = A22 - A21 T  (the Schur complement),  Y = S^-1,
        A^-1 = [[X11 + T Y U, -T Y], [-Y U, Y]].
    Six GEMMs of half size per level (2 n^3 flops in all, the flops of getrf + getri), written straight
    into the quadrants of the result (views with a leading dimension, no copies); leaves of at most
    `base` rows inverted in one launch each by the Gauss-Jordan kernel of this library on the GPU
    (sem_dense_inverse_small, partial pivoting within the leaf; rocSOLVER took ~130 us per 64^2 leaf,
    tools/pivot_probe.py --profile), by torch's pivoted LU on the host.  No pivoting across the split: every leading block
    must be regular, which holds for the diagonally dominated pivot blocks of the interface sweep and is
    not assumed -- the caller checks A X - I (velocity_solve.pivot_inverse) and falls back to a pivoted
    LU when it misses.  A singular leaf gives non-finite entries, never an exception."""
    return _block_inv(A, base, torch.empty_like(A) if out is None else out)


def small_inverse_into(A, X):
    """X = A^-1 for one n x n float64 CUDA block, n <= 64, through the library's one-workgroup
    Gauss-Jordan kernel (sem_dense_inverse_small); A and X may be row-major views with a leading
    dimension.  Non-finite entries for a singular block."""
    from . import _lib
    n = A.shape[-1]
    if A.stride(1) != 1 or X.stride(1) != 1:
        raise ValueError("small_inverse_into needs unit column stride")
    lib = _lib.load()
    _lib.check(lib.sem_dense_inverse_small(C.c_void_p(A.data_ptr()), A.stride(0), C.c_void_p(X.data_ptr()),
                                           X.stride(0), n,
                                           C.c_void_p(torch.cuda.current_stream(A.device).cuda_stream)))
    return X


def _block_inv(A, base, X):
    n = A.shape[-1]
    if A.is_cuda and n <= 64:   # the one-launch Gauss-Jordan leaf
        return small_inverse_into(A, X)
    if n <= base:
        X.copy_(torch.linalg.inv_ex(A)[0])
        return X
    h = _split(n)
    A11, A12, A21, A22 = A[:h, :h], A[:h, h:], A[h:, :h], A[h:, h:]
    X11, X12, X21, X22 = X[:h, :h], X[:h, h:], X[h:, :h], X[h:, h:]
    _block_inv(A11, base, X11)
    T = X11 @ A12
    U = A21 @ X11
    _block_inv(torch.addmm(A22, A21, T, alpha=-1.0), base, X22)
    torch.addmm(X12, T, X22, beta=0.0, alpha=-1.0, out=X12)
    torch.addmm(X21, X22, U, beta=0.0, alpha=-1.0, out=X21)
    X11.addmm_(X12, U, alpha=-1.0)
    return X
