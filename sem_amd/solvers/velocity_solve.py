"""Device direct solve of the Navier-Stokes velocity Jacobian.

Replaces the reference's host SuperLU of the 2N x 2N velocity Jacobian
(NavierStokes_Solver.py:176-192: `bmat` -> Dirichlet rows -> `splu`, then `lu.solve` twice per
Schur-complement matvec) with a static condensation that fits the structured SEM mesh:

* Node lines in the x-major numbering (SEM.py:110) are either *interface* lines x = L P
  (L = 0..N_ex) or one of the P-1 *interior* lines of an element column.  The operators couple a
  node only to nodes of the same line (y direction) and of the same element column (x direction),
  so the interior lines of column e couple to each other and to interface lines e and e+1 only.
* `sem_velocity_blocks` (HIP, sem_amd/csrc/ns_velocity.hip) writes the pieces: one dense block
  A_II per element column ((P-1) 2 N_y unknowns), the dense interface-line blocks D, and the
  diagonal line-to-line couplings.
* Factor: batched pivoted LU of the A_II blocks (rocSOLVER through torch), W = A_II^-1 A_IB, the
  interface Schur complement S = A_BB - A_BI W (block tridiagonal over the N_ex+1 interface lines,
  blocks of 2 N_y), and its block-LU (block Thomas) with explicit inverses of the pivot blocks.
* Solve: interior forward solve, the interface sweep (block cyclic reduction: ~3 batched launches
  per level, log2(N_ex+1) levels; or block Thomas, 2 N_ex dependent GEMVs), interior back substitution.

Everything is device memory: cfg3 (32^2, P = 8) holds 3.3 GB of A_II factors, cfg4 (48^2, P = 8)
11 GB, well inside one MI355X's 288 GB.  The algebra runs on any torch device, so the
condensation itself is unit-tested on CPU against SciPy's sparse solve
(tests/test_velocity_solve.py); the block assembly needs the GPU.
"""
import contextlib
import math
import os
import time

import torch

from ..device import no_gc
from ..tracing import phase

GEMV_LDS_DOUBLES = 8192   # sem_block_gemv stages S m operand doubles in LDS (include/sem_ops.h)


# rocSOLVER's strided-batched getrf/getri (sem_amd/linalg.py) in place of torch's pointer-array batched
# path (hipblasDgetrfBatched, faulty on this stack); SEM_STRIDED_INV=0 selects torch's for A/B runs
_STRIDED = os.environ.get("SEM_STRIDED_INV", "1") != "0"


def _inverse(A):
    """Inverse of a batch and its per-block LU status (0 = regular; None when the route reports none):
    rocSOLVER strided-batched on the GPU, else torch.linalg.inv_ex; on a getrf workspace-allocation failure
    the batch is halved."""
    if _STRIDED and A.is_cuda and A.dim() == 3:
        from .. import linalg
        if linalg.available():
            try:
                return linalg.strided_inverse(A)
            except RuntimeError:
                if A.shape[0] == 1:
                    raise
                h = A.shape[0] // 2
                (x1, i1), (x2, i2) = _inverse(A[:h]), _inverse(A[h:])
                return torch.cat((x1, x2)), torch.cat((i1, i2))
    try:
        return torch.linalg.inv_ex(A)
    except RuntimeError as e:
        if "ALLOC_FAILED" not in str(e) or A.dim() < 3 or A.shape[0] == 1:
            raise
    out = torch.empty_like(A)
    info = torch.empty(A.shape[0], dtype=torch.int32, device=A.device)
    step = max(1, A.shape[0] // 2)
    for i in range(0, A.shape[0], step):
        out[i:i + step], info[i:i + step] = _inverse(A[i:i + step])
    return out, info


def _bad_blocks(A, X):
    """Blocks whose computed inverse misses: max |A X - I| above 8 n^2 eps |A|max |X|max.  Entry (i, j)
    of A X sums n products bounded by |A|max |X|max, so forming it rounds by at most n eps n |A| |X|,
    and a backward-stable inverse adds an error of the same order: the bound is purely relative, it
    accepts ill-conditioned blocks (large |A| |X|) and rejects a wrong inverse, whose residual is of
    order |A| |X| itself."""
    E = A @ X
    E.diagonal(dim1=-2, dim2=-1).sub_(1.0)
    n = A.shape[-1]
    scale = A.abs().amax(dim=(-2, -1)) * X.abs().amax(dim=(-2, -1))
    tol = 8.0 * n * n * torch.finfo(A.dtype).eps * scale
    return torch.nonzero(~(E.abs().amax(dim=(-2, -1)) <= tol)).flatten()


def batched_inverse(A, max_batch=None, sample=8):
    """Inverses of a batch of blocks, sliced and spot-checked.

    torch's batched LU on this ROCm stack is faulty (tools/inv_repro.py on MI355X,
    profiles/r03/inv/inv_repro_mi355x.txt): on seeded, well-conditioned, contiguous 121^2 blocks
    (U(-1, 1) + n I) torch.linalg.inv, inv_ex, lu_factor + lu_solve and solve -- every route goes through
    hipblasDgetrfBatched (pointer-array batched) -- return correct inverses (residual 2e-15) in batches up
    to 512 and wrong ones without an error at 1024 (16 of 1024 blocks) and 4096 (950 of 4096); 242^2
    blocks fail their workspace allocation from batch 256 on.  The caller is not involved (fresh
    contiguous tensors, no views).  rocSOLVER's strided-batched getrf + getri on the same blocks
    (sem_amd/linalg.py) is correct at every batch measured (up to 16384 blocks of 242^2, residual 5e-15)
    and runs at 5.2 TFLOP/s there against 0.17 for the sliced torch route, so it is the GPU path
    (_inverse).  Either way the batch is inverted in slices of max_batch (4096 strided, 128 through torch)
    and each slice is spot-checked through the residual A X - I of `sample` blocks (its first, its last
    and evenly spaced ones); a slice is checked in full when its sample misses, when the LU reports a
    singular pivot for any block or when any block of the result is not finite (both checks read the batch
    once, cheap beside getri); a block that misses is inverted again on its own (then by a solve against the
    identity) before giving up."""
    if A.dim() < 3:
        return batched_inverse(A[None], max_batch, sample)[0]
    if max_batch is None:   # rocSOLVER's strided path measured correct up to 16384 blocks; torch's to 512
        max_batch = 4096 if (_STRIDED and A.is_cuda) else 128
    out = torch.empty_like(A)
    for i in range(0, A.shape[0], max_batch):
        a = A[i:i + max_batch]
        x, info = _inverse(a)
        nb = a.shape[0]
        pick = torch.linspace(0, nb - 1, min(nb, sample), device=a.device).round().long().unique()
        suspect = ~x.isfinite().all(dim=-1).all(dim=-1)
        if info is not None:
            suspect |= info != 0
        full = _bad_blocks(a[pick], x[pick]).numel() > 0 or bool(suspect.any())
        for j in (_bad_blocks(a, x).tolist() if full else []):
            xj = torch.linalg.inv(a[j])
            if _bad_blocks(a[j:j + 1], xj[None]).numel():
                eye = torch.eye(a.shape[-1], dtype=a.dtype, device=a.device)
                xj = torch.linalg.solve(a[j], eye)
                if _bad_blocks(a[j:j + 1], xj[None]).numel():
                    raise RuntimeError("velocity solve: an interior block could not be inverted accurately")
            x[j] = xj
        out[i:i + max_batch] = x
    return out


_PIVOT_INV = os.environ.get("SEM_PIVOT_INV", "block")  # "block" | "lu" | "inv" | "strided" (sweep pivots)


def _pivot_ok(A, X, r):
    """|A (X r) - r| within 8 n^2 eps |A| |X| |r| (the relative bound of _bad_blocks, on one probe)."""
    n = A.shape[-1]
    res = (A @ (X @ r) - r).abs().max()
    tol = 8.0 * n * n * torch.finfo(A.dtype).eps * A.abs().max() * X.abs().max() * r.abs().max()
    return bool(res <= tol)


def pivot_inverse(A):
    """Inverse of one large pivot block of the interface sweep (m x m, m up to 3,074 at cfg5).

    Default ("block"): the GEMM-recursive inverse (sem_amd/linalg.py block_inverse) -- rocSOLVER's
    getrf runs at 2.4 TFLOP/s on one 3,074^2 block against 55 for a GEMM of that size on MI355X
    (tools/pivot_probe.py, profiles/r03/cfg5/pivot_probe.jsonl), and the 129 sequential pivots of the cfg5
    block-Thomas sweep spent ~3.5 s there.  The recursion does not pivot across its splits, so the result
    is checked on a random probe vector (|A (X r) - r| within 8 n^2 eps |A| |X| |r|); on a miss
    E = A X - I is formed (one GEMM) and the inverse refined by one Newton step X <- X - X E when E is a
    contraction (row sums below 1/2: the error squares), checked again; otherwise -- a leading block
    singular or badly conditioned -- it is replaced by the pivoted route.
    "lu": LU factorisation and a triangular solve against the identity (getrf + getrs), checked on a
    random probe vector; a miss falls back to the checked batched path (batched_inverse)."""
    n = A.shape[-1]
    g = torch.Generator(device=A.device).manual_seed(7)
    r = torch.rand(n, dtype=A.dtype, device=A.device, generator=g) - 0.5
    if _PIVOT_INV == "block" and n > 64:
        from ..linalg import block_inverse
        X = block_inverse(A)
        if _pivot_ok(A, X, r):
            return X
        E = A @ X
        E.diagonal().sub_(1.0)
        if bool(E.abs().sum(dim=1).max() < 0.5):
            X = X - X @ E
            if _pivot_ok(A, X, r):
                return X
    if _PIVOT_INV == "strided":
        return batched_inverse(A)
    if _PIVOT_INV == "inv":
        X = torch.linalg.inv(A)
    else:
        LU, piv = torch.linalg.lu_factor(A)
        X = torch.linalg.lu_solve(LU, piv, torch.eye(n, dtype=A.dtype, device=A.device))
    if not _pivot_ok(A, X, r):
        return batched_inverse(A)
    return X


def fused_thomas_operators(Dinv, S_lo, Uh):
    """Operators of the fused block-Thomas solve of a block-tridiagonal system with lines 0..n-1, from its
    factors (explicit pivot-block inverses Dinv (n, m, m), lower blocks S_lo (n-1, m, m), Uh_L = Dinv_L S_up_L):
    z_0 = D_0 g_0, z_L = F_L [g_L; z_{L-1}] with F_L = [D_L | -D_L S_lo[L-1]] (m x 2m), back z_L -= Uh_L z_{L+1}:
    one GEMV per line and direction, each operator read once (the m x 2m GEMV runs at 5.7 TB/s at cfg5's
    m = 3,074, tools/gemv_probe.py)."""
    n, m = Dinv.shape[0], Dinv.shape[1]
    F = torch.empty((max(n - 1, 0), m, 2 * m), dtype=Dinv.dtype, device=Dinv.device)
    if n > 1:
        F[:, :, :m] = Dinv[1:]
    for L in range(n - 1):
        F[L, :, m:] = -(Dinv[L + 1] @ S_lo[L])
    return Dinv[0].clone(), F, Uh


_SWEEP_GEMV = os.environ.get("SEM_SWEEP_GEMV", "hip")   # "hip": sem_gemv_rows; "torch": rocBLAS (A/B)


def _gemv(A, x, y, alpha=1.0, beta=0.0):
    """y = alpha A x + beta y for a row-major operator: the library's streaming GEMV on the GPU
    (sem_gemv_rows: 5+ TB/s on operators read once, where rocBLAS's gemvt streamed 3.6), torch elsewhere."""
    if A.is_cuda and _SWEEP_GEMV == "hip" and A.dtype == torch.float64 and A.stride(1) == 1 and x.stride(0) == 1 \
            and y.stride(0) == 1:
        import ctypes as C
        from .. import _lib
        lib = _lib.load()
        _lib.check(lib.sem_gemv_rows(A.shape[0], A.shape[1], alpha, C.c_void_p(A.data_ptr()), A.stride(0),
                                     C.c_void_p(x.data_ptr()), beta, C.c_void_p(y.data_ptr()),
                                     C.c_void_p(torch.cuda.current_stream(A.device).cuda_stream)))
        return y
    if beta == 0.0:
        torch.mv(A, x, out=y)
        if alpha != 1.0:
            y.mul_(alpha)
    else:
        y.mul_(beta).addmv_(A, x, alpha=alpha)
    return y


def _gemv2(p0, p1, alpha=1.0, beta=0.0):
    """Two independent GEMVs (A, x, y) of equal row count in one launch (sem_gemv_rows2); torch elsewhere."""
    (A0, x0, y0), (A1, x1, y1) = p0, p1
    ok = lambda A, x, y: (A.is_cuda and A.dtype == torch.float64 and A.stride(1) == 1  # noqa: E731
                          and x.stride(0) == 1 and y.stride(0) == 1)
    if _SWEEP_GEMV == "hip" and A0.shape[0] == A1.shape[0] and ok(A0, x0, y0) and ok(A1, x1, y1):
        import ctypes as C
        from .. import _lib
        lib = _lib.load()
        v = C.c_void_p
        _lib.check(lib.sem_gemv_rows2(A0.shape[0], alpha, beta, A0.shape[1], v(A0.data_ptr()), A0.stride(0),
                                      v(x0.data_ptr()), v(y0.data_ptr()), A1.shape[1], v(A1.data_ptr()), A1.stride(0),
                                      v(x1.data_ptr()), v(y1.data_ptr()),
                                      v(torch.cuda.current_stream(A0.device).cuda_stream)))
        return
    _gemv(A0, x0, y0, alpha, beta)
    _gemv(A1, x1, y1, alpha, beta)


def twisted_thomas_operators(S_diag, S_up, S_lo, inv=None):
    """Operators of the twisted ("burn at both ends") block-Thomas solve of a block-tridiagonal system with
    lines 0..n-1 (n >= 3; diagonal S_diag, S_up[L]: row L <- L+1, S_lo[L]: row L+1 <- L): elimination from
    line 0 down to k-1 and from line n-1 up to k+1 (k = n // 2), the two chains meeting at line k.
      top     Dt_0 = S_diag[0], UhT_L = Dt_L^-1 S_up[L], Dt_{L+1} = S_diag[L+1] - S_lo[L] UhT_L
      bottom  Et_{n-1} = S_diag[n-1], UhB_L = Et_L^-1 S_lo[L-1], Et_{L-1} = S_diag[L-1] - S_up[L-1] UhB_L
      middle  M = S_diag[k] - S_lo[k-1] UhT_{k-1} - S_up[k] UhB_{k+1}
    Fused forward operators as in fused_thomas_operators: FT_L = [Dt_L^-1 | -Dt_L^-1 S_lo[L-1]] (L = 1..k-1),
    FB_L = [Et_L^-1 | -Et_L^-1 S_up[L]] (L = k+1..n-2), FM = [M^-1 | -M^-1 S_lo[k-1] | -M^-1 S_up[k]]; the
    same 3 m^2 doubles per line as the one-ended sweep (plus m^2 for the middle) and the same pivot
    inverses, but the two chains run side by side (twisted_thomas_solve): n + 1 dependent steps, not 2 n - 1."""
    inv = inv or pivot_inverse
    n, m = S_diag.shape[0], S_diag.shape[1]
    if n < 3:
        raise ValueError("the twisted sweep needs at least 3 lines")
    k = n // 2
    z = dict(dtype=S_diag.dtype, device=S_diag.device)
    FT, UhT = torch.empty((k - 1, m, 2 * m), **z), torch.empty((k, m, m), **z)
    FB, UhB = torch.empty((n - 2 - k, m, 2 * m), **z), torch.empty((n - 1 - k, m, m), **z)
    Dt = S_diag[0]
    for L in range(k):
        if L > 0:
            Dt = S_diag[L] - S_lo[L - 1] @ UhT[L - 1]
        Di = inv(Dt)
        if L == 0:
            D0 = Di
        else:
            FT[L - 1, :, :m] = Di
            FT[L - 1, :, m:] = -(Di @ S_lo[L - 1])
        UhT[L] = Di @ S_up[L]
    for L in range(n - 1, k, -1):
        i = L - (k + 1)
        Et = S_diag[L] if L == n - 1 else S_diag[L] - S_up[L] @ UhB[i + 1]
        Ei = inv(Et)
        if L == n - 1:
            E0 = Ei
        else:
            FB[i, :, :m] = Ei
            FB[i, :, m:] = -(Ei @ S_up[L])
        UhB[i] = Ei @ S_lo[L - 1]
    Mi = inv(S_diag[k] - S_lo[k - 1] @ UhT[k - 1] - S_up[k] @ UhB[0])
    FM = torch.cat((Mi, -(Mi @ S_lo[k - 1]), -(Mi @ S_up[k])), dim=1)
    return k, D0, E0, FT, FB, FM, UhT, UhB


def twisted_thomas_solve(op, g):
    """x = S^-1 g from twisted_thomas_operators (g: (n, m), not modified).  Work rows W[L] = [g_L | s_L | t_L]:
    a top line's slot s_L holds z_{L-1}, a bottom line's holds w_{L+1}, the middle line k holds z_{k-1} and
    w_{k+1} (s_k, t_k), so every forward GEMV reads one contiguous 2m (middle: 3m) vector and writes its result
    straight into the slot of the next line of its chain; each step of the two chains is ONE launch
    (sem_gemv_rows2), the back substitution updates the slots in place.  Stream-capturable."""
    k, D0, E0, FT, FB, FM, UhT, UhB = op
    n, m = g.shape[0], g.shape[1]
    W = torch.empty((n, 3 * m), dtype=g.dtype, device=g.device)
    W[:, :m] = g
    top = lambda L: W[L + 1, m:2 * m]                                        # noqa: E731  z_L, then x_L
    bot = lambda L: W[k, 2 * m:] if L == k + 1 else W[L - 1, m:2 * m]        # noqa: E731  w_L, then x_L
    x_k = torch.empty(m, dtype=g.dtype, device=g.device)
    # forward: step 0 (D0 g_0, E0 g_{n-1}), then the chains side by side
    _gemv2((D0, g[0], top(0)), (E0, g[n - 1], bot(n - 1)))
    steps_t, steps_b = list(range(1, k)), list(range(n - 2, k, -1))
    for j in range(max(len(steps_t), len(steps_b))):
        pt = (FT[steps_t[j] - 1], W[steps_t[j], :2 * m], top(steps_t[j])) if j < len(steps_t) else None
        pb = (FB[steps_b[j] - (k + 1)], W[steps_b[j], :2 * m], bot(steps_b[j])) if j < len(steps_b) else None
        if pt and pb:
            _gemv2(pt, pb)
        else:
            _gemv(*(pt or pb))
    _gemv(FM, W[k], x_k)
    # back: x_L = z_L - UhT_L x_{L+1} (L = k-1 .. 0) beside x_L = w_L - UhB_L x_{L-1} (L = k+1 .. n-1)
    steps_t, steps_b = list(range(k - 1, -1, -1)), list(range(k + 1, n))
    xt = lambda L: x_k if L == k else top(L)                                 # noqa: E731
    for j in range(max(len(steps_t), len(steps_b))):
        Lt = steps_t[j] if j < len(steps_t) else None
        Lb = steps_b[j] if j < len(steps_b) else None
        pt = (UhT[Lt], xt(Lt + 1), top(Lt)) if Lt is not None else None
        pb = (UhB[Lb - (k + 1)], x_k if Lb - 1 == k else bot(Lb - 1), bot(Lb)) if Lb is not None else None
        if pt and pb:
            _gemv2(pt, pb, alpha=-1.0, beta=1.0)
        else:
            _gemv(*(pt or pb), alpha=-1.0, beta=1.0)
    x = torch.empty((n, m), dtype=g.dtype, device=g.device)   # sem_nested_solve reads x_B as a packed (n, m) array
    x[:k] = W[1:k + 1, m:2 * m]
    x[k] = x_k
    x[k + 1] = W[k, 2 * m:]
    x[k + 2:] = W[k + 1:n - 1, m:2 * m]
    return x


def twisted_thomas_solve_mat(op, g):
    """X = S^-1 G for a block right-hand side G (n, m, c) from twisted_thomas_operators: the recurrences of
    twisted_thomas_solve with GEMMs (the strip solve's coupling solutions X0, X1 from the same factors as its sweep,
    strip_solve.StripLineSolver._sweep_factor; ADVICE r4: no second, one-ended set of pivot inverses)."""
    k, D0, E0, FT, FB, FM, UhT, UhB = op
    n, m = g.shape[0], g.shape[1]
    z = [None] * n                    # z_L (top chain, L < k), w_L (bottom chain, L > k)
    z[0] = D0 @ g[0]
    for L in range(1, k):
        z[L] = FT[L - 1, :, :m] @ g[L] + FT[L - 1, :, m:] @ z[L - 1]
    z[n - 1] = E0 @ g[n - 1]
    for L in range(n - 2, k, -1):
        i = L - (k + 1)
        z[L] = FB[i, :, :m] @ g[L] + FB[i, :, m:] @ z[L + 1]
    x = torch.empty_like(g)
    x[k] = FM[:, :m] @ g[k] + FM[:, m:2 * m] @ z[k - 1] + FM[:, 2 * m:] @ z[k + 1]
    for L in range(k - 1, -1, -1):
        x[L] = z[L] - UhT[L] @ x[L + 1]
    for L in range(k + 1, n):
        x[L] = z[L] - UhB[L - (k + 1)] @ x[L - 1]
    return x


def fused_thomas_solve(D0, F, Uh, g):
    """x = S^-1 g from fused_thomas_operators (g: (n, m), not modified).  W[L] = [g_L | z_{L-1}]: the
    forward GEMV of line L reads one contiguous 2m vector and writes z_L straight into W[L+1]'s second
    half, so no copy sits in the chain; no host synchronisation (stream-capturable)."""
    n, m = g.shape[0], g.shape[1]
    W = torch.empty((n + 1, 2 * m), dtype=g.dtype, device=g.device)
    W[:n, :m] = g
    _gemv(D0, g[0], W[1, m:])
    for L in range(1, n):
        _gemv(F[L - 1], W[L], W[L + 1, m:])
    z = W[1:, m:]                       # z_L at row L
    for L in range(n - 2, -1, -1):
        _gemv(Uh[L], z[L + 1], z[L], alpha=-1.0, beta=1.0)
    return z.contiguous()             # sem_nested_solve reads x_B as a packed (n, m) array


class VelocityJacobianSolver:
    """x = J^-1 b for the velocity Jacobian J of one linearisation, J given by its condensation pieces."""

    def __init__(self, P, nex, ney, device, interior="nested", sweep="auto", ncomp=2):
        """ncomp: unknowns per node -- 2 for the velocity pair [u | v], 1 for a scalar operator
        (the convection-diffusion Jacobian, or the pressure stiffness of the Schur preconditioner).
        interior: elimination of the element-column interiors ("nested" static condensation, or
        one dense block per column: "lu" factors, "inverse" explicit inverses).  sweep: solve of the
        block-tridiagonal interface system ("cr": block cyclic reduction, about 2 log2(N_ex) batched
        launches; "thomas": block Thomas, 2 N_ex sequential steps, a third of CR's factorisation flops and
        fewer bytes per solve; "auto": CR up to m = 2048 interface unknowns per line, Thomas above --
        measured: CR's solve is faster at cfg3/cfg4 (m = 514 / 770), its factorisation dominates cfg5's
        (m = 3074: 4.6 s of 8.3 s, profiles/r03/cfg5/))."""
        if P < 1 or nex < 1 or ney < 1:
            raise ValueError("bad mesh")
        if interior not in ("nested", "lu", "inverse"):
            raise ValueError("interior must be 'nested', 'lu' or 'inverse'")
        if sweep not in ("cr", "thomas", "auto"):
            raise ValueError("sweep must be 'cr', 'thomas' or 'auto'")
        if ncomp not in (1, 2):
            raise ValueError("ncomp must be 1 or 2")
        self.sweep, self.ncomp = sweep, ncomp
        self.P, self.nex, self.ney = P, nex, ney
        self.NY, self.NX = ney * P + 1, nex * P + 1
        self.m = ncomp * self.NY
        self.nI = (P - 1) * self.m
        if sweep == "auto":
            sweep = self.sweep = "cr" if self.m <= 2048 else "thomas"
        self.device = torch.device(device)
        self.interior = interior
        self.factored = False
        # SEM_PROFILE_FACTOR=1: per-phase wall times of the factorisation (device-synchronised)
        self.profile = os.environ.get("SEM_PROFILE_FACTOR", "") == "1"
        self.timing = {}
        # edge Schur systems up to this size are inverted densely (pivoted); larger ones by block LU.  On the
        # GPU every size takes the checked block LU (its block-Thomas sweeps read (N_ey+1) 3 ne1^2 doubles per
        # column instead of n_e^2: 48.5 -> ~15 us per edge step at cfg4, profiles/r03/vel48/); a column
        # whose block LU fails the check still gets the pivoted dense inverse
        self.edge_dense_max = 0 if self.device.type == "cuda" else 1024
        # edge solve of the block-LU path on the GPU: "auto" keeps the block-Thomas factors (sem_nested_solve's
        # ABI-9 form: O(N_ey ne1^2) doubles per column read per solve instead of the n_e^2 of the dense
        # inverse -- 1.5 MB instead of 64 MB per cfg5 column); "dense" keeps the dense inverse
        self.edge_solve = "auto"
        self._edge_thomas = False
        # HIP nested solves: "coupled" (ABI 11: the interface right-hand side from the forward element step's
        # T = Xi b_i and the edge values, sem_nested_iface_rhs; the back substitution T -= Xi A_iB x_B from the
        # same work arrays, sem_nested_back_solve) or "full" (the ABI-10 path: y_I formed, then a second nested
        # solve of b_I - A_IB x_B through Xi)
        self.nested_back = os.environ.get("SEM_NESTED_BACK", "coupled")
        # block-Thomas interface sweep on the GPU: "twisted" (two-ended: the chains from line 0 and from line N_ex
        # meet in the middle, one launch per step of both, twisted_thomas_solve) or "single" (one-ended, the
        # fused forward operators of fused_thomas_operators)
        self.sweep_form = os.environ.get("SEM_SWEEP_FORM", "twisted")
        # one step of iterative refinement x += J^-1 (b - J x), gated at factor time by the factor's measured
        # backward error (check_refinement).  The nested condensation eliminates the element-
        # column interiors first, with no pivoting across that split: where a column interior is far worse
        # conditioned than J (kappa 2.0e6 against kappa(J) = 9.8e3 for the one-component Pe = 1000 operator on
        # 2 x 2 elements, P = 6) the solve's backward error is ~1e-11 where SuperLU's pivoting gives ~4e-17
        # (NavierStokes_Solver.py:184); one refinement step brings it to 3e-17 (tools/backward_error_probe.py)
        self._apply = None
        self._amax = None
        self.refine = False
        self.refine_eta = None

    @contextlib.contextmanager
    def _phase(self, name):
        if not self.profile:
            yield
            return
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        yield
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.timing[name] = self.timing.get(name, 0.0) + time.perf_counter() - t0

    # ------------------------------------------------------------------ assembly
    def empty_blocks(self, with_interior=True):
        """Zeroed storage for the pieces, in sem_velocity_blocks' layout."""
        P, nex, m, nI = self.P, self.nex, self.m, self.nI
        z = dict(dtype=torch.float64, device=self.device)
        return dict(AII=torch.zeros((nex, nI, nI), **z) if P > 1 and with_interior else None,
                    D=torch.zeros((nex + 1, m, m), **z),
                    aIB=torch.zeros((nex, P - 1, 2, m), **z) if P > 1 else None,
                    aBI=torch.zeros((nex, 2, P - 1, m), **z) if P > 1 else None,
                    E=torch.zeros((nex, m), **z), F=torch.zeros((nex, m), **z))

    # ------------------------------------------------------------------ factorisation
    def interior_bytes(self):
        """Bytes of the dense A_II blocks of the whole mesh."""
        return self.nex * self.nI * self.nI * 8

    def factor_from(self, fill, budget_bytes=24 << 30):
        """Assemble the dense-interior layout (sem_velocity_blocks: fill(blocks, cols) with blocks["AII"]
        holding the dense interiors of element columns cols = (c0, c1)) and factor it.  Used by the "lu" /
        "inverse" interior variants and by tests; the default nested interior assembles the condensed
        layout directly (factor_mesh -> factor_condensed)."""
        if self.P > 1 and self.nex * self.nI * self.nI * 8 > budget_bytes:
            raise ValueError("the dense column interiors exceed the memory budget: use factor_mesh (condensed)")
        blocks = self.empty_blocks()
        fill(blocks, (0, self.nex))
        return self.factor(blocks.pop("AII"), **blocks)

    # ------------------------------------------------------------------ condensed assembly (ABI 7)
    # The nested condensation straight from its pieces: the HIP kernel (sem_condensed_blocks) writes
    # every element's interior block A_ii, its couplings A_ie / A_ei to the column's horizontal edges, and
    # the block-tridiagonal edge operator A_ee -- no dense column interior A_II (9 GB per column at cfg5).
    # With Xi = A_ii^-1 and the edge Schur complement S_e = A_ee - A_ei Xi A_ie, the interface coupling
    # of a column, A_BI A_II^-1 A_IB, is
    #     C = A_Bi Xi A_iB + Z_B S_e^-1 Z_e,  Z_e = A_eB - A_ei Xi A_iB,  Z_B = A_Be - A_Bi Xi A_ie,
    # where A_iB / A_Bi couple an element's interior to the interface nodes at the same y (group G_n of
    # the interface unknowns: (s, c, nP + j)) and A_eB / A_Be couple an edge to the interface nodes at its
    # y (group H_k: (s, c, kP)).  Z_e is block-banded (the columns of G_n live on edges n, n+1; those of H_k
    # on edge k), so V = S_e^-1 Z_e and Z_B V are batched products of thin blocks: O(n_e m ne1) per
    # column instead of the O(n_I^2 m) of A_II^-1 A_IB.
    def condensed_empty(self, ncols):
        """Zeroed per-column condensed pieces of ncols element columns (sem_condensed_blocks layout)."""
        P, ney, nc = self.P, self.ney, self.ncomp
        ne1 = nc * (P - 1)
        ni = ne1 * (P - 1)
        z = dict(dtype=torch.float64, device=self.device)
        return dict(Aii=torch.zeros((ncols, ney, ni, ni), **z), Aie=torch.zeros((ncols, ney, ni, 2 * ne1), **z),
                    Aei=torch.zeros((ncols, ney, 2 * ne1, ni), **z), Aed=torch.zeros((ncols, ney + 1, ne1, ne1), **z),
                    Aeu=torch.zeros((ncols, ney, ne1, ne1), **z), Ael=torch.zeros((ncols, ney, ne1, ne1), **z))

    def condense_dense(self, AII):
        """The condensed pieces of dense column interiors AII (ncols, nI, nI): the layout
        sem_condensed_blocks writes, taken from the dense blocks (CPU tests, interior="nested" factor())."""
        self._nested_index()
        ncols, ney, ne1 = AII.shape[0], self.ney, self._ne1
        pi, pe, pel = self._pi, self._pe, self._pe_el
        e = torch.arange(ncols, device=AII.device)[:, None, None, None]
        out = dict(Aii=AII[e, pi[None, :, :, None], pi[None, :, None, :]],
                   Aie=AII[e, pi[None, :, :, None], pel[None, :, None, :]],
                   Aei=AII[e, pel[None, :, :, None], pi[None, :, None, :]])
        Aee = AII[e[:, :, 0], pe[None, :, None], pe[None, None, :]].view(ncols, ney + 1, ne1, ney + 1, ne1)
        k = torch.arange(ney + 1, device=AII.device)
        out["Aed"] = Aee[:, k, :, k, :].permute(1, 0, 2, 3).contiguous()
        out["Aeu"] = Aee[:, k[:-1], :, k[1:], :].permute(1, 0, 2, 3).contiguous()
        out["Ael"] = Aee[:, k[1:], :, k[:-1], :].permute(1, 0, 2, 3).contiguous()
        return out

    def factor_mesh(self, mesh, budget_bytes=24 << 30, **kw):
        """Assemble on the device (HIP) and factor the Jacobian with the coefficients kw (the keywords of
        device.Mesh.condensed_blocks / velocity_blocks): the condensed layout for the nested interior,
        the dense column interiors for the "lu" / "inverse" variants."""
        kw = dict(kw, ncomp=self.ncomp)
        if self.P > 1 and self.interior == "nested":
            return self.factor_condensed(lambda b, cols: mesh.condensed_blocks(b, cols=cols, **kw), budget_bytes)
        return self.factor_from(lambda b, cols: mesh.velocity_blocks(b, cols=cols, **kw), budget_bytes)

    def _alloc_factor(self):
        """Storage of the nested factor.  On the GPU the blocks are kept column-major (the layout
        sem_nested_solve reads) and the row-major names are transposed views of it."""
        nex, ney, ne1 = self.nex, self.ney, self._ne1
        ni, n_e = self._pi.shape[1], self._pe.numel()
        z = dict(dtype=torch.float64, device=self.device)
        self._edge_thomas = n_e > self.edge_dense_max and ne1 <= 32 and (
            self.edge_solve == "thomas" or (self.edge_solve == "auto" and self.device.type == "cuda"))
        shapes = ((nex, ney, ni, ni), (nex, ney, 2 * ne1, ni), (nex, ney, ni, 2 * ne1), (nex, n_e, n_e))
        if self._edge_thomas:   # block-Thomas factors of the edge Schur complement instead of its inverse
            shapes = shapes[:3]
            Et = [torch.empty(sh, **z) for sh in ((nex, ney + 1, ne1, ne1), (nex, ney, ne1, ne1), (nex, ney, ne1, ne1))]
            self._EtT = tuple(Et)                                   # row-major blocks (ABI 10)
            self._Ed, self._El, self._Eu = Et
        if self.device.type == "cuda":
            T = [torch.empty(s[:-2] + (s[-1], s[-2]), **z) for s in shapes]
            if self._edge_thomas:
                T.append(None)
            self._hipT = tuple(T)
            self._Xi, self._Aei, self._Yie, self._Se_inv = (None if t is None else t.transpose(-1, -2) for t in T)
            # ABI 11: Xi A_iB and A_ei Xi A_iB of every element (by-products of the coupling products), so the
            # back substitution's element step reads 2 ne1 columns instead of Xi's ni (sem_nested_back_solve)
            # and A_Bi Xi A_ie, so the forward half forms the interface right-hand side without the element
            # values y_i (sem_nested_iface_rhs)
            G = 2 * ne1
            self._hipB = (torch.empty((nex, ney, G, ni), **z), torch.empty((nex, ney, G, G), **z),
                          torch.empty((nex, ney, G, G), **z))
            self._XiB, self._AXB, self._ABY = (t.transpose(-1, -2) for t in self._hipB)
        else:
            self._hipT = self._hipB = self._XiB = self._AXB = self._ABY = None
            self._Xi, self._Aei, self._Yie, self._Se_inv = [torch.empty(s, **z) for s in shapes] + (
                [None] if self._edge_thomas else [])

    def factor_condensed(self, fill, budget_bytes=24 << 30, pieces=None, line=None, chunk_cols=None):
        """Factor from condensed pieces: fill(blocks, cols) writes the pieces of element columns cols and the
        interface pieces (sem_condensed_blocks), a chunk of columns at a time within budget_bytes of work
        memory; or pieces / line given directly (CPU, from condense_dense)."""
        P, nex, ney, m = self.P, self.nex, self.ney, self.m
        self._nested_index()
        ne1 = self._ne1
        ni, n_e = ne1 * (P - 1), (ney + 1) * ne1
        per_col = 8 * (3 * ney * ni * ni + 6 * ney * ni * 2 * ne1 + 3 * n_e * n_e + 4 * n_e * 2 * m
                       + 2 * ney * 2 * ne1 * 2 * m + 3 * (2 * m) ** 2)
        chunk = nex if pieces is not None else max(1, min(nex, int(budget_bytes // per_col)))
        if chunk_cols:
            chunk = int(chunk_cols)
        self._alloc_factor()
        S_diag = S_up = S_lo = None
        for c0 in range(0, nex, chunk):
            c1 = min(nex, c0 + chunk)
            if pieces is None:
                with self._phase("fill"):
                    if line is None:
                        line = self.empty_blocks(with_interior=False)
                    blk = dict(line)
                    blk.update(self.condensed_empty(c1 - c0))
                    fill(blk, (c0, c1))
            else:
                blk = dict(line)
                blk.update(pieces)
            if S_diag is None:   # every fill writes the interface pieces in full: take them from the first
                aIB, aBI = blk["aIB"], blk["aBI"]
                S_diag = blk["D"].clone()
                S_up, S_lo = torch.diag_embed(blk["E"]), torch.diag_embed(blk["F"])
            C = self._condense_chunk(blk, aIB, aBI, c0, c1)
            del blk
            with self._phase("coupling"):
                S_diag[c0:c1] -= C[:, :m, :m]
                S_diag[c0 + 1:c1 + 1] -= C[:, m:, m:]
                S_up[c0:c1] -= C[:, :m, m:]
                S_lo[c0:c1] -= C[:, m:, :m]
                del C
        self._nested_finish()
        self.W = None
        self.aBI, self.aIB = aBI, aIB
        with self._phase("sweep_factor"):
            self._sweep_factor(S_diag, S_up, S_lo)

    def _group_perm(self):
        """Interface-unknown order of the coupling products: groups G_0..G_{ney-1} ((s, c, j) each), then
        H_0..H_ney ((s, c) each); returns, for every line-layout index s m + c N_y + gy, its group index."""
        if getattr(self, "_gperm", None) is None:
            P, ney, nc, NY, m = self.P, self.ney, self.ncomp, self.NY, self.m
            dev = self.device
            s = torch.arange(2, device=dev)
            c = torch.arange(nc, device=dev)
            n = torch.arange(ney, device=dev)
            j = torch.arange(1, P, device=dev)
            k = torch.arange(ney + 1, device=dev)
            g_line = (s[None, :, None, None] * m + c[None, None, :, None] * NY + n[:, None, None, None] * P
                      + j[None, None, None, :]).reshape(-1)
            h_line = (s[None, :, None] * m + c[None, None, :] * NY + k[:, None, None] * P).reshape(-1)
            lines = torch.cat((g_line, h_line))
            inv = torch.empty_like(lines)
            inv[lines] = torch.arange(lines.numel(), device=dev)
            self._gperm = inv
        return self._gperm

    def _condense_chunk(self, blk, aIB, aBI, c0, c1):
        """Factor pieces of columns [c0, c1) into the solver's arrays and their interface coupling
        C = A_BI A_II^-1 A_IB (cc, 2m, 2m) in the line layout (s m + c N_y + gy)."""
        P, ney, nc, NY, m = self.P, self.ney, self.ncomp, self.NY, self.m
        ne1 = self._ne1
        ni, n_e, G, cc = ne1 * (P - 1), (ney + 1) * ne1, 2 * ne1, c1 - c0
        dev, f64 = self.device, torch.float64
        Aii, Aie = blk["Aii"].view(cc, ney, ni, ni), blk["Aie"].view(cc, ney, ni, G)
        Aei = blk["Aei"].view(cc, ney, G, ni)
        with self._phase("inv_element"):
            Xi = batched_inverse(Aii.reshape(-1, ni, ni)).view(cc, ney, ni, ni)
        with self._phase("edge_schur"):
            Yie = Xi @ Aie
            Cee = Aei @ Yie                                   # (cc, ney, 2 ne1, 2 ne1): rows / cols edges n, n+1
            Sd = blk["Aed"].view(cc, ney + 1, ne1, ne1).clone()
            Sd[:, :-1] -= Cee[:, :, :ne1, :ne1]
            Sd[:, 1:] -= Cee[:, :, ne1:, ne1:]
            Su = blk["Aeu"].view(cc, ney, ne1, ne1) - Cee[:, :, :ne1, ne1:]
            Sl = blk["Ael"].view(cc, ney, ne1, ne1) - Cee[:, :, ne1:, :ne1]
            del Cee
        with self._phase("inv_edge"):
            Se_inv, fac = self._blocktri_inverse(Sd, Su, Sl, factors=True)
        self._Xi[c0:c1], self._Yie[c0:c1], self._Aei[c0:c1] = Xi, Yie, Aei
        if self._edge_thomas and fac is None:   # a column needed the pivoted dense inverse: dense edge solve
            self._edge_to_dense(c0)
        if self._edge_thomas:
            self._Ed[c0:c1], self._El[c0:c1], self._Eu[c0:c1] = fac[0], Sl, fac[1]
        else:
            self._Se_inv[c0:c1] = Se_inv
        with self._phase("coupling_pieces"):
            eye_c = torch.eye(nc, dtype=f64, device=dev)
            eye_j = torch.eye(P - 1, dtype=f64, device=dev)
            gy_i = (torch.arange(ney, device=dev)[:, None] * P + torch.arange(1, P, device=dev)[None, :]).reshape(-1)
            gy_e = torch.arange(ney + 1, device=dev) * P
            vIB = aIB[c0:c1].view(cc, P - 1, 2, nc, NY)          # [e, l, s, c, gy]
            vBI = aBI[c0:c1].view(cc, 2, P - 1, nc, NY)          # [e, s, l, c, gy]
            # A_iB[e, n, (l c j), (s c' j')] and A_Bi[e, n, (s c j), (l c' j')], diagonal in (c, j)
            a = vIB[..., gy_i].view(cc, P - 1, 2, nc, ney, P - 1)
            AiB = torch.einsum("elscnj,cd,jk->enlcjsdk", a, eye_c, eye_j).reshape(cc, ney, ni, G)
            b = vBI[..., gy_i].view(cc, 2, P - 1, nc, ney, P - 1)
            ABi = torch.einsum("eslcnj,cd,jk->enscjldk", b, eye_c, eye_j).reshape(cc, ney, G, ni)
            # A_eB[e, k, (l c), (s c')], A_Be[e, k, (s c), (l c')]
            AeB = torch.einsum("elsck,cd->eklcsd", vIB[..., gy_e], eye_c).reshape(cc, ney + 1, ne1, 2 * nc)
            ABe = torch.einsum("eslck,cd->ekscld", vBI[..., gy_e], eye_c).reshape(cc, ney + 1, 2 * nc, ne1)
            XiB = Xi @ AiB                                     # (cc, ney, ni, G)
            C_GG = ABi @ XiB                                   # (cc, ney, G, G)
            ZeG = -(Aei @ XiB)                                 # rows: edges n, n+1
            ZBG = -(ABi @ Yie)                                 # cols: edges n, n+1
            if self._XiB is not None:   # kept for sem_nested_back_solve / sem_nested_iface_rhs (ABI 11)
                self._XiB[c0:c1] = XiB
                torch.neg(ZeG, out=self._AXB[c0:c1])
                torch.neg(ZBG, out=self._ABY[c0:c1])
            del AiB, XiB, Xi, Yie
        with self._phase("coupling_products"):
            # V = S_e^-1 Z_e in the group order of the columns
            SeW = Se_inv.unfold(2, G, ne1).permute(0, 2, 1, 3)           # (cc, ney, n_e, 2 ne1): edges n, n+1
            VG = SeW @ ZeG                                                # (cc, ney, n_e, G)
            SeH = Se_inv.view(cc, n_e, ney + 1, ne1).permute(0, 2, 1, 3)  # (cc, ney+1, n_e, ne1)
            VH = SeH @ AeB                                                # (cc, ney+1, n_e, 2 nc)
            V = torch.cat((VG.permute(0, 2, 1, 3).reshape(cc, n_e, ney * G),
                           VH.permute(0, 2, 1, 3).reshape(cc, n_e, (ney + 1) * 2 * nc)), dim=2)
            del VG, VH, SeW, SeH
            # C = Z_B V (+ A_Bi Xi A_iB on the G diagonal blocks), rows in group order
            Vw = V.unfold(1, G, ne1).transpose(-1, -2)                    # (cc, ney, 2 ne1, 2m): rows edges n, n+1
            CG = ZBG @ Vw                                                 # (cc, ney, G, 2m)
            CH = ABe @ V.view(cc, ney + 1, ne1, 2 * m)                    # (cc, ney+1, 2 nc, 2m)
            del Vw, V
            Cg = torch.cat((CG.reshape(cc, ney * G, 2 * m), CH.reshape(cc, (ney + 1) * 2 * nc, 2 * m)), dim=1)
            del CG, CH
            Cv = Cg[:, :ney * G, :ney * G].view(cc, ney, G, ney, G)
            n = torch.arange(ney, device=dev)
            Cv[:, n, :, n, :] += C_GG.permute(1, 0, 2, 3)
            inv = self._group_perm()
            return Cg[:, inv][:, :, inv]

    def _blocktri_inverse(self, Sd, Su, Sl, factors=False):
        """Dense inverse of block-tridiagonal matrices (batched over columns): diagonal blocks Sd (cc, nb, b, b),
        upper Su[k] (row block k, column block k+1), lower Sl[k] (row k+1, column k).  Block LU with pivoted
        inverses of the pivot blocks, then the block-Thomas solve against the identity; the result is
        checked through its residual S X - I (block-tridiagonal times dense: cheap) and a column whose
        elimination without inter-block pivoting lost accuracy is inverted densely instead.
        factors=True: returns (X, (Dinv, Uh)) -- the block-Thomas factors (inverse pivot blocks and
        Dinv_k Su_k) the checked inverse was built from, or None when they are absent (a dense inverse)
        or when a column failed the check."""
        cc, nb, b = Sd.shape[0], Sd.shape[1], Sd.shape[2]
        n = nb * b
        if n <= self.edge_dense_max:   # small edge systems: one pivoted dense inverse per column
            S = self._blocktri_dense(Sd, Su, Sl)
            X = batched_inverse(S)
            return (X, None) if factors else X
        # pivot-block inverses without raising: a singular or ill-conditioned pivot shows in the final check
        inv = lambda A: torch.linalg.inv_ex(A)[0]  # noqa: E731
        Dinv = torch.empty_like(Sd)
        Uh = torch.empty_like(Su)
        Dinv[:, 0] = inv(Sd[:, 0])
        for k in range(1, nb):
            Uh[:, k - 1] = Dinv[:, k - 1] @ Su[:, k - 1]
            Dinv[:, k] = inv(Sd[:, k] - Sl[:, k - 1] @ Uh[:, k - 1])
        X = self._blocktri_apply_identity(Dinv, Uh, Sl)
        res = self._blocktri_residual(Sd, Su, Sl, X)
        bad = torch.nonzero(~(res <= 8.0 * n * n * torch.finfo(Sd.dtype).eps)).flatten().tolist()
        if bad:
            S = self._blocktri_dense(Sd[bad], Su[bad], Sl[bad])
            X[bad] = batched_inverse(S)
        if factors:
            return X, (None if bad else (Dinv, Uh))
        return X

    @staticmethod
    def _blocktri_apply_identity(Dinv, Uh, Sl):
        """S^-1 from the block-Thomas factors of S (batched over columns)."""
        cc, nb, b = Dinv.shape[0], Dinv.shape[1], Dinv.shape[2]
        n = nb * b
        dev, f64 = Dinv.device, Dinv.dtype
        X = torch.zeros((cc, nb, b, n), dtype=f64, device=dev)
        # forward: Z_k = Dinv_k (I_k - Sl_{k-1} Z_{k-1}); Z_k is zero beyond column block k
        X[:, 0, :, :b] = Dinv[:, 0]
        for k in range(1, nb):
            w = k * b
            R = -(Sl[:, k - 1] @ X[:, k - 1, :, :w])
            X[:, k, :, :w] = Dinv[:, k] @ R
            X[:, k, :, w:w + b] = Dinv[:, k]
        # back: X_k = Z_k - Uh_k X_{k+1}
        for k in range(nb - 2, -1, -1):
            X[:, k] -= Uh[:, k] @ X[:, k + 1]
        return X.view(cc, n, n)

    def _edge_to_dense(self, c0):
        """Leave the block-Thomas edge form (a column of chunk c0.. failed its check): dense inverses for the
        columns factored so far, rebuilt from their checked factors, and the dense form from here on."""
        nex, n_e = self.nex, self._pe.numel()
        SeT = torch.empty((nex, n_e, n_e), dtype=torch.float64, device=self.device)
        self._Se_inv = SeT.transpose(-1, -2)
        for a in range(0, c0, 8):
            b = min(c0, a + 8)
            self._Se_inv[a:b] = self._blocktri_apply_identity(self._Ed[a:b], self._Eu[a:b], self._El[a:b])
        if self._hipT is not None:
            self._hipT = self._hipT[:3] + (SeT,)
        self._edge_thomas = False
        self._Ed = self._El = self._Eu = self._EtT = None

    @staticmethod
    def _blocktri_dense(Sd, Su, Sl):
        cc, nb, b = Sd.shape[0], Sd.shape[1], Sd.shape[2]
        S = torch.zeros((cc, nb, b, nb, b), dtype=Sd.dtype, device=Sd.device)
        k = torch.arange(nb, device=Sd.device)
        S[:, k, :, k, :] = Sd.permute(1, 0, 2, 3)
        S[:, k[:-1], :, k[1:], :] = Su.permute(1, 0, 2, 3)
        S[:, k[1:], :, k[:-1], :] = Sl.permute(1, 0, 2, 3)
        return S.view(cc, nb * b, nb * b)

    @staticmethod
    def _blocktri_residual(Sd, Su, Sl, X):
        """max |S X - I| / (|S|max |X|max) per column, S block tridiagonal."""
        cc, nb, b = Sd.shape[0], Sd.shape[1], Sd.shape[2]
        Xb = X.view(cc, nb, b, nb * b)
        R = Sd @ Xb
        R[:, :-1] += Su @ Xb[:, 1:]
        R[:, 1:] += Sl @ Xb[:, :-1]
        Rv = R.view(cc, nb * b, nb * b)
        Rv.diagonal(dim1=-2, dim2=-1).sub_(1.0)
        smax = torch.maximum(torch.maximum(Sd.abs().amax(dim=(1, 2, 3)), Su.abs().amax(dim=(1, 2, 3))),
                             Sl.abs().amax(dim=(1, 2, 3))) if nb > 1 else Sd.abs().amax(dim=(1, 2, 3))
        return Rv.abs().amax(dim=(1, 2)) / (smax * X.abs().amax(dim=(1, 2)))

    def _interface_coupling(self, aBI, W):
        """C[e, s, r, t, k] = sum_l aBI[e, s, l, r] W[e, l, r, t, k]: A_BI A_II^-1 A_IB per column."""
        nc, P, m = W.shape[0], self.P, self.m
        Wr = W.view(nc, P - 1, m, 2, m)
        C = torch.zeros((nc, 2, m, 2, m), dtype=torch.float64, device=self.device)
        for li in range(P - 1):
            C += aBI[:, :, li, :, None, None] * Wr[:, None, li]
        return C

    def factor(self, AII, D, aIB, aBI, E, F):
        """Condense and factor.  AII is consumed (its storage is reused for the LU factors)."""
        P, nex, m = self.P, self.nex, self.m
        if P > 1 and self.interior == "nested":   # the condensed path, pieces taken from the dense blocks
            pieces = self.condense_dense(AII)
            del AII
            return self.factor_condensed(None, pieces=pieces, line=dict(D=D, aIB=aIB, aBI=aBI, E=E, F=F))
        if P > 1:
            # dense A_IB (nex, nI, 2m): rows (l, r), column block s holds aIB[e, l, s, r] on its diagonal
            AIB = torch.diag_embed(aIB).permute(0, 1, 3, 2, 4).reshape(nex, self.nI, 2 * m)
            LU, piv, info = torch.linalg.lu_factor_ex(AII)
            del AII
            if int(info.max().item()) > 0:
                raise RuntimeError("velocity Jacobian: singular interior block")
            W = torch.linalg.lu_solve(LU, piv, AIB)
            del AIB
            C = self._interface_coupling(aBI, W)   # A_BI W for both interface lines
            S_diag = D.clone()
            S_diag[:-1] -= C[:, 0, :, 0, :]
            S_diag[1:] -= C[:, 1, :, 1, :]
            S_up = torch.diag_embed(E) - C[:, 0, :, 1, :]
            S_lo = torch.diag_embed(F) - C[:, 1, :, 0, :]
            del C
            if self.interior == "inverse":
                eye = torch.eye(self.nI, dtype=torch.float64, device=self.device).expand(nex, -1, -1)
                self.Ainv = torch.linalg.lu_solve(LU, piv, eye)
                del LU, piv
                self.LU = self.piv = None
            elif self.interior == "lu":
                self.LU, self.piv = LU, piv
            self.W = W.view(nex, self.nI, 2, m)
            self.aBI, self.aIB = aBI, aIB
        else:
            S_diag, S_up, S_lo = D, torch.diag_embed(E), torch.diag_embed(F)
        self._sweep_factor(S_diag, S_up, S_lo)

    def _sweep_factor(self, S_diag, S_up, S_lo):
        nex, m = self.nex, self.m
        if self.sweep == "cr":
            self._cr_factor(S_diag, S_up, S_lo)
            self.factored = True
            return
        self._tw = None
        if self.sweep_form == "twisted" and self.device.type == "cuda" and nex + 1 >= 3:
            # two-ended block Thomas (round 4): the same operator bytes, half the dependent launches
            self._tw = twisted_thomas_operators(S_diag, S_up, S_lo)
            self._th = self.Dinv = self.Uh = self.S_lo = None
            self.factored = True
            return
        # block Thomas on the interface lines: Dt[0] = S_diag[0], Uh[L] = Dt[L]^-1 S_up[L],
        # Dt[L+1] = S_diag[L+1] - S_lo[L] Uh[L]; explicit (pivoted) inverses of the pivot blocks
        Dinv = torch.empty((nex + 1, m, m), dtype=torch.float64, device=self.device)
        Uh = torch.empty((nex, m, m), dtype=torch.float64, device=self.device)
        Dt = S_diag[0]
        for L in range(nex + 1):
            if L > 0:
                Dt = S_diag[L] - S_lo[L - 1] @ Uh[L - 1]
            Dinv[L] = pivot_inverse(Dt)
            if L < nex:
                Uh[L] = Dinv[L] @ S_up[L]
        self.Dinv, self.Uh, self.S_lo = Dinv, Uh, S_lo
        self._th = None
        if self.device.type == "cuda" and os.environ.get("SEM_THOMAS_FUSED", "1") != "0":
            self._th = fused_thomas_operators(Dinv, S_lo, Uh)
            self.Dinv = self.S_lo = None
        self.factored = True

    # ------------------------------------------------------------------ interface sweep: cyclic reduction
    # Block cyclic reduction of the block-tridiagonal interface system (rows L = 0..N_ex, diagonal
    # blocks B_L = S_diag[L], couplings A_L = S_lo[L-1] to row L-1 and C_L = S_up[L] to row L+1).
    # Each level eliminates every other remaining row j with the explicit inverse of its pivot block:
    # a kept row i with neighbours l < i < r takes
    #     alpha_i = -A_i B_l^-1, gamma_i = -C_i B_r^-1,  B_i += alpha_i C_l + gamma_i A_r,
    #     A_i <- alpha_i A_l, C_i <- gamma_i C_r,        g_i += alpha_i g_l + gamma_i g_r,
    # and back substitution recovers x_j = B_j^-1 g_j - (B_j^-1 A_j) x_l - (B_j^-1 C_j) x_r.  Missing
    # neighbours get zero blocks, so every level is one batched product per direction: the solve is
    # ~3 launches per level and log2(N_ex + 1) levels, against the 2 N_ex dependent steps of Thomas.
    def _cr_factor(self, S_diag, S_up, S_lo):
        n, m = S_diag.shape[0], S_diag.shape[1]
        dev, f64 = self.device, torch.float64
        B = S_diag.clone()
        A = torch.zeros_like(B)
        C = torch.zeros_like(B)
        if n > 1:
            A[1:] = S_lo
            C[:-1] = S_up
        rows = torch.arange(n, device=dev)
        self._cr = []
        while rows.numel() > 1:
            keep, elim = rows[0::2].contiguous(), rows[1::2].contiguous()   # index arrays of sem_block_gemv
            k = keep.numel()
            # neighbours of the kept rows (-1: none) and of the eliminated rows (always kept rows)
            left = torch.full((k,), -1, dtype=torch.long, device=dev)
            right = torch.full((k,), -1, dtype=torch.long, device=dev)
            left[1:] = elim[:k - 1]
            right[:elim.numel()] = elim
            Binv = batched_inverse(B[elim])
            hasl, hasr = left >= 0, right >= 0
            zl, zr = left.clamp(min=0), right.clamp(min=0)
            pos = torch.full((n,), -1, dtype=torch.long, device=dev)
            pos[elim] = torch.arange(elim.numel(), device=dev)
            Bl = torch.where(hasl[:, None, None], Binv[pos[zl].clamp(min=0)], torch.zeros((), dtype=f64, device=dev))
            Br = torch.where(hasr[:, None, None], Binv[pos[zr].clamp(min=0)], torch.zeros((), dtype=f64, device=dev))
            alpha = -(A[keep] @ Bl)
            gamma = -(C[keep] @ Br)
            B[keep] += alpha @ C[zl] + gamma @ A[zr]
            # back-substitution operator of the eliminated rows: [B^-1 | -B^-1 A | -B^-1 C]
            back = torch.cat((Binv, -(Binv @ A[elim]), -(Binv @ C[elim])), dim=2)
            nA, nC = alpha @ A[zl], gamma @ C[zr]
            A[keep], C[keep] = nA, nC
            fwd = torch.cat((alpha, gamma), dim=2)
            # gather index of [g_l; g_r] for the kept rows (missing neighbours read row 0, times zero)
            # back substitution reads [g_j; x_l; x_r]; a missing right neighbour (zero block) reads x_l
            e = elim.numel()
            br = torch.cat((keep[1:], keep[-1:]))[:e]
            br_hip = torch.cat((keep[1:], keep.new_full((1,), -1)))[:e]   # sem_block_gemv: -1 = absent
            self._cr.append((keep, fwd.contiguous(), torch.stack((zl, zr)), elim, back.contiguous(),
                             torch.stack((elim, keep[:e], br)),
                             torch.stack((left, right)).contiguous(), torch.stack((elim, keep[:e], br_hip)).contiguous()))
            rows = keep
        self._cr_top = (rows.contiguous(), batched_inverse(B[rows]).contiguous())

    def _cr_solve(self, g):
        """x = S^-1 g for the interface system; g (N_ex + 1, m) is overwritten.  On the GPU every level
        is one sem_block_gemv launch per direction (HIP, HBM-bound on the level's operators)."""
        if self.device.type == "cuda":
            return self._cr_solve_hip(g)
        for keep, fwd, idx, *_ in self._cr:
            gl = g[idx.reshape(-1)].view(2, keep.numel(), -1).permute(1, 0, 2).reshape(keep.numel(), -1, 1)
            g.index_add_(0, keep, torch.bmm(fwd, gl)[..., 0])
        top, Tinv = self._cr_top
        x = torch.zeros_like(g)
        x[top] = torch.bmm(Tinv, g[top][..., None])[..., 0]
        for _, _, _, elim, back, idx, *_ in reversed(self._cr):
            rhs = torch.cat((g[idx[0]], x[idx[1]], x[idx[2]]), dim=1)[..., None]
            x[elim] = torch.bmm(back, rhs)[..., 0]
        return x

    def _block_gemv(self, M, srcs, xrow, y, yrow, acc):
        """y[yrow[b]] (+)= sum_s M[b][:, s m:(s+1) m] srcs[s][xrow[s][b]]: one sem_block_gemv launch (a batched
        torch GEMV for operands beyond the kernel's LDS staging)."""
        import ctypes as C
        from .. import _lib
        m, S = y.shape[1], len(srcs)
        if not (M.is_contiguous() and xrow.is_contiguous() and yrow.is_contiguous()
                and xrow.dtype == yrow.dtype == torch.int64 and tuple(M.shape) == (yrow.numel(), m, S * m)
                and tuple(xrow.shape) == (S, yrow.numel())):
            raise ValueError("sem_block_gemv: operator / index layout")
        if S * m > GEMV_LDS_DOUBLES:   # operands beyond the kernel's LDS staging (cfg5's CR: m = 3074): batched GEMV
            rhs = torch.cat([torch.where((r >= 0)[:, None], t[r.clamp(min=0)], 0.0) for t, r in zip(srcs, xrow)],
                            dim=1)
            out = torch.bmm(M, rhs[..., None])[..., 0]
            if acc:
                y[yrow] += out
            else:
                y[yrow] = out
            return
        lib = _lib.load()
        P = C.c_void_p
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        src = (P * S)(*(P(t.data_ptr()) for t in srcs))
        ld = (C.c_int64 * S)(*(t.stride(0) for t in srcs))
        _lib.check(lib.sem_block_gemv(yrow.numel(), m, S, P(M.data_ptr()), src, ld, P(xrow.data_ptr()),
                                      P(y.data_ptr()), y.stride(0), P(yrow.data_ptr()), int(acc), stream))

    def _cr_solve_hip(self, g):
        x = torch.zeros_like(g)
        gemv = self._block_gemv
        for keep, fwd, _, _, _, _, fx, _ in self._cr:
            gemv(fwd, (g, g), fx, g, keep, True)
        top, Tinv = self._cr_top
        gemv(Tinv, (g,), top.reshape(1, -1).contiguous(), x, top.contiguous(), False)
        for _, _, _, elim, back, _, _, bx in reversed(self._cr):
            gemv(back, (g, x, x), bx, x, elim, False)
        return x

    # ------------------------------------------------------------------ nested interior (default)
    # Inside one element column the interior unknowns split again: the interiors of its elements
    # (y nodes strictly inside element n, on all P-1 interior lines: 2 (P-1)^2 unknowns) couple only
    # to the horizontal element edges y = nP, (n+1)P of the same lines.  So A_II is eliminated in
    # two levels -- batched inverses of the small element-interior blocks, then one dense block of
    # the column's edge unknowns (2 (P-1)(N_ey+1)) -- the classical static condensation of SEM
    # element interiors.  A column solve then reads ~100x fewer bytes than a dense A_II^-1.
    def _nested_index(self):
        P, ney, NY, m = self.P, self.ney, self.NY, self.m
        dev = self.device
        l = torch.arange(1, P, device=dev)
        c = torch.arange(self.ncomp, device=dev)
        col = lambda ll, cc, gy: (ll - 1) * m + cc * NY + gy  # noqa: E731  column-interior ordering
        # element interiors: (n, l, c, j) with gy = nP + j, j = 1..P-1
        n = torch.arange(ney, device=dev)
        j = torch.arange(1, P, device=dev)
        pi = col(l[None, :, None, None], c[None, None, :, None], n[:, None, None, None] * P + j[None, None, None, :])
        self._pi = pi.reshape(ney, -1)                                  # (ney, 2 (P-1)^2)
        # edges: (k, l, c) with gy = kP, k = 0..ney
        k = torch.arange(ney + 1, device=dev)
        pe = col(l[None, :, None], c[None, None, :], k[:, None, None] * P)
        self._ne1 = self.ncomp * (P - 1)                                # unknowns per edge row k
        self._pe = pe.reshape(-1)                                       # (n_e,)
        self._pe_el = torch.cat((pe[:-1].reshape(ney, -1), pe[1:].reshape(ney, -1)), dim=1)  # edges k=n, n+1

    def _nested_finish(self):
        if self.device.type == "cuda":   # column-major blocks for sem_nested_solve (ns_condense.hip)
            if getattr(self, "_hipT", None) is None:
                self._hipT = tuple(None if t is None else t.transpose(-1, -2).contiguous() for t in
                                   (self._Xi, self._Aei, self._Yie, self._Se_inv))
            self._pi, self._pe = self._pi.contiguous(), self._pe.contiguous()

    def _nested_solve(self, R, cols=slice(None)):
        """A_II^-1 R for every column (or the columns `cols`) at once; R (columns, nI, k)."""
        nex, ney, ne1 = R.shape[0], self.ney, self._ne1
        k = R.shape[-1]
        Ri = R[:, self._pi]                                             # (nex, ney, ni, k)
        Re = R[:, self._pe].clone()                                     # (nex, n_e, k)
        Ti = self._Xi[cols] @ Ri
        Cn = self._Aei[cols] @ Ti                                       # (nex, ney, 2 ne1, k)
        Rv = Re.view(nex, ney + 1, ne1, k)
        Rv[:, :-1] -= Cn[:, :, :ne1]
        Rv[:, 1:] -= Cn[:, :, ne1:]
        if self._edge_thomas:
            Ye = self._edge_thomas_solve(Re, cols)
        else:
            Ye = self._Se_inv[cols] @ Re                                # (nex, n_e, k)
        Yv = Ye.view(nex, ney + 1, ne1, k)
        Yi = Ti - self._Yie[cols] @ torch.cat((Yv[:, :-1], Yv[:, 1:]), dim=2)
        Y = torch.empty_like(R)
        Y[:, self._pi] = Yi
        Y[:, self._pe] = Ye
        return Y

    def _edge_thomas_solve(self, Re, cols=slice(None)):
        """S_e^-1 Re from the block-Thomas factors (the torch form of cond_edge_thomas_kernel)."""
        Ed, El, Eu = self._Ed[cols], self._El[cols], self._Eu[cols]
        nex, nb, b = Ed.shape[0], Ed.shape[1], Ed.shape[2]
        R = Re.view(nex, nb, b, -1)
        Z = torch.empty_like(R)
        Z[:, 0] = Ed[:, 0] @ R[:, 0]
        for k in range(1, nb):
            Z[:, k] = Ed[:, k] @ (R[:, k] - El[:, k - 1] @ Z[:, k - 1])
        for k in range(nb - 2, -1, -1):
            Z[:, k] -= Eu[:, k] @ Z[:, k + 1]
        return Z.view(Re.shape)

    # ------------------------------------------------------------------ solve
    def _hip_nested(self):
        """Descriptor and work arrays of sem_nested_solve / sem_interface_rhs (built once)."""
        if getattr(self, "_nd", None) is None:
            from .. import _lib
            nex, ney, P, m = self.nex, self.ney, self.P, self.m
            ni, ne1 = self._pi.shape[1], self._ne1
            z = dict(dtype=torch.float64, device=self.device)
            if getattr(self, "_work", None) is None:
                self._work = (torch.empty(nex * ney * ni, **z), torch.empty(nex * ney * 2 * ne1, **z),
                              torch.empty(nex * (ney + 1) * ne1, **z), torch.empty((nex, self.nI), **z),
                              torch.empty((nex + 1, m), **z), torch.empty(nex * 2 * m, **z))
            T, Cw, Ye, _, _, Pw = self._work
            p = lambda t: t.data_ptr()  # noqa: E731
            XiT, AeiT, YieT, SeT = self._hipT
            Et = self._EtT if self._edge_thomas else (None, None, None)   # ABI 9: Se = NULL -> block Thomas
            if self._edge_thomas:   # ABI 10: the sweep computes the edge offsets; they must be _pe's
                kk = torch.arange(ney + 1, device=self.device)[:, None]
                q = torch.arange(ne1, device=self.device)[None, :]
                want = (q // self.ncomp) * m + (q % self.ncomp) * self.NY + kk * P
                if not torch.equal(want.reshape(-1), self._pe):
                    raise RuntimeError("nested solve: edge offsets differ from the block-Thomas sweep's layout")
            q = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
            hb = self._hipB if getattr(self, "_hipB", None) is not None else (None, None, None)
            self._nd = _lib.SemNestedDesc(P, nex, ney, self.ncomp, self.NY, p(XiT), p(AeiT), p(YieT), q(SeT),
                                          p(self._pi), p(self._pe), p(T), p(Cw), p(Ye), *(q(t) for t in Et),
                                          *(q(t) for t in hb), p(Pw))
        return self._nd

    def _own_rhs(self, g, B):
        """Hook of the strip-partitioned solve (strip_solve.py): drop the right-hand side of an interface
        line this part does not own.  Whole mesh: nothing to do."""

    def _iface_solve(self, g):
        """The interface system S xB = g (overwrites g)."""
        if self.sweep == "cr":
            return self._cr_solve(g)
        if getattr(self, "_tw", None) is not None:
            return twisted_thomas_solve(self._tw, g)
        if getattr(self, "_th", None) is not None:
            return fused_thomas_solve(*self._th, g)
        # block Thomas with the pivot blocks' explicit inverses: 2 GEMVs per line forward, 1 back
        z = g
        z[0] = self.Dinv[0] @ g[0]
        for L in range(1, self.nex + 1):
            z[L] = self.Dinv[L] @ (g[L] - self.S_lo[L - 1] @ z[L - 1])
        for L in range(self.nex - 1, -1, -1):
            z[L] -= self.Uh[L] @ z[L + 1]
        return z

    def _solve_lines_hip(self, B):
        """_solve_lines on the GPU with the nested interior solves and the interface right-hand side
        as HIP kernels (sem_amd/csrc/ns_condense.hip): 3 + 1 + CR + 3 launches, no gathers or copies."""
        import ctypes as C
        from .. import _lib
        lib = _lib.load()
        P, nex, m, NX = self.P, self.nex, self.m, self.NX
        if not (B.is_contiguous() and tuple(B.shape) == (NX, m) and B.dtype == torch.float64):
            raise ValueError("line array must be a contiguous float64 (NX, m) tensor")
        d = self._hip_nested()
        _, _, _, yI, g, _ = self._work
        st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        v = C.c_void_p
        b1 = B.data_ptr() + 8 * m   # line e P + 1: first interior line of column e
        coupled = bool(d.XiB) and self.nested_back == "coupled"
        with phase("vsolve.nested_fwd"):
            if coupled:   # ABI 11: element and edge steps, then g from T and the edge values (no y_I formed)
                _lib.check(lib.sem_nested_iface_rhs(C.byref(d), v(b1), P * m, v(B.data_ptr()), m,
                                                    v(self.aBI.data_ptr()), v(yI.data_ptr()), self.nI,
                                                    v(g.data_ptr()), st))
            else:
                _lib.check(lib.sem_nested_solve(C.byref(d), v(b1), P * m, None, None, v(yI.data_ptr()), self.nI,
                                                st))
                _lib.check(lib.sem_interface_rhs(P, nex, m, v(B.data_ptr()), m, v(self.aBI.data_ptr()),
                                                 v(yI.data_ptr()), self.nI, v(g.data_ptr()), st))
            self._own_rhs(g, B)
        with phase("vsolve.iface_solve"):
            xB = self._iface_solve(g)
        out = torch.empty((NX, m), dtype=torch.float64, device=self.device)
        out[0::P] = xB
        # back substitution x_I = A_II^-1 (b_I - A_IB x_B): by default from the forward solve's work arrays and
        # Xi A_iB (ABI 11; nested_back = "full" re-solves with Xi, the ABI-10 path, for A/B)
        back = lib.sem_nested_back_solve if coupled else lib.sem_nested_solve
        with phase("vsolve.nested_back"):
            _lib.check(back(C.byref(d), v(b1), P * m, v(self.aIB.data_ptr()), v(xB.data_ptr()),
                            v(out.data_ptr() + 8 * m), P * m, st))
        return out

    # ------------------------------------------------------------------ iterative refinement
    def set_operator(self, apply_lines, amax=None):
        """apply_lines(X) -> J X on (NX, m) line arrays (the matrix-free Jacobian apply of the solver that owns
        this factor); amax(t) -> max |t| over every part (a partitioned solve reduces over the ranks)."""
        self._apply = apply_lines
        self._amax = amax if amax is not None else (lambda t: float(t.abs().max()))

    def check_refinement(self, tau=None, seed=17):
        """Measure the factor's normwise backward error eta = ||J x - b|| / (||J|| ||x|| + ||b||) (max norms) on a
        seeded probe, ||J|| estimated from below by ||J s|| for a random sign vector s (so eta is over-estimated),
        and turn on one refinement step per solve when eta > tau (SEM_REFINE_ETA, default 1e-13; 0 refines
        always, inf never).  Every part of a partitioned solve takes the same decisions (reduced norms).  A
        non-finite eta (a singular or overflowing factor block) raises RuntimeError instead of passing as "no
        refinement needed" (max(0, nan) is 0).  Returns eta."""
        if self._apply is None:
            raise RuntimeError("set_operator() first")
        if tau is None:
            tau = float(os.environ.get("SEM_REFINE_ETA", "1e-13"))
        # probe vectors drawn over the GLOBAL lines and sliced: on a partition, a shared line's entries must be equal
        # on both ranks (the strip solve's contract); per-rank draws made them differ and the residual of the
        # inconsistent right-hand side read as a backward error of 1e-4 at cfg5 (a false refinement)
        l0, l1, NXg = self._probe_lines()
        g = torch.Generator(device=self.device).manual_seed(seed)
        b = (torch.rand((NXg, self.m), dtype=torch.float64, device=self.device, generator=g) * 2 - 1)[l0:l1].contiguous()
        sgn = torch.sign(torch.rand((NXg, self.m), dtype=torch.float64, device=self.device, generator=g)
                         - 0.5)[l0:l1].contiguous()
        self.refine = False
        nJ = self._amax(self._apply(sgn))
        probes = {0: b}

        def probe(k):   # probe k: right-hand side k (0: the one above; more drawn on demand, same generator)
            if k not in probes:
                probes[k] = (torch.rand((NXg, self.m), dtype=torch.float64, device=self.device, generator=g) * 2
                             - 1)[l0:l1].contiguous()
            bk = probes[k]
            x = self._solve_lines(bk)
            return self._amax(bk - self._apply(x)) / (nJ * self._amax(x) + self._amax(bk))

        eta = probe(0)
        if not math.isfinite(eta):
            raise RuntimeError(f"velocity factor: non-finite backward error on the probe ({eta}): a singular or "
                               "overflowing pivot block")
        self.refine_eta = eta
        self.refine = eta > tau
        return eta

    def _probe_lines(self):
        """(first, end, count) of this solver's lines among all lines of the mesh: the whole mesh here."""
        return 0, self.NX, self.NX

    def _solve_lines(self, B):
        """x = J^-1 b with b, x as (NX, 2 NY) line arrays (every line: u then v); with `refine` set, one step of
        iterative refinement on the matrix-free Jacobian apply."""
        X = self._solve_lines_once(B)
        if self.refine:
            X = X + self._solve_lines_once(B - self._apply(X))
        return X

    def _solve_lines_once(self, B):
        P, nex, m, NX = self.P, self.nex, self.m, self.NX
        if (self.device.type == "cuda" and P > 1 and self.interior == "nested"
                and getattr(self, "hip_nested", True)):
            return self._solve_lines_hip(B)
        g = B[0::P].clone()                                    # interface lines (nex+1, m)
        if P > 1:
            bI = B[:-1].reshape(nex, P, m)[:, 1:, :].reshape(nex, self.nI, 1)
            if self.interior == "nested":
                yI = self._nested_solve(bI)
            elif self.interior == "inverse":
                yI = torch.bmm(self.Ainv, bI)
            else:
                yI = torch.linalg.lu_solve(self.LU, self.piv, bI)
            yIr = yI.view(nex, P - 1, m)
            g[:-1] -= (self.aBI[:, 0] * yIr).sum(1)
            g[1:] -= (self.aBI[:, 1] * yIr).sum(1)
        self._own_rhs(g, B)
        xB = self._iface_solve(g)
        out = torch.empty((NX, m), dtype=torch.float64, device=self.device)
        out[0::P] = xB
        if P > 1:
            if self.interior == "nested":   # x_I = A_II^-1 (b_I - A_IB x_B); A_IB is diagonal per line
                rI = bI.view(nex, P - 1, m) - (self.aIB[:, :, 0, :] * xB[:-1, None, :]
                                                + self.aIB[:, :, 1, :] * xB[1:, None, :])
                xI = self._nested_solve(rI.reshape(nex, self.nI, 1))
            else:
                xI = yI.view(nex, self.nI) - (torch.bmm(self.W[:, :, 0, :], xB[:-1, :, None])
                                              + torch.bmm(self.W[:, :, 1, :], xB[1:, :, None]))[..., 0]
            out[:-1].view(nex, P, m)[:, 1:, :] = xI.view(nex, P - 1, m)
        return out

    def capture(self):
        """Capture the solve (about 3 (N_ex+1) + 10 launches) in a hipGraph: a Schur-complement
        matvec then costs the kernels, not the Python and launch overhead of that many small ops.
        Returns False (and the solve stays eager) if the device libraries refuse the capture."""
        if self.device.type != "cuda" or not self.factored:
            return False
        if self.P > 1 and self.interior == "lu":
            return False   # the batched LU solve (rocSOLVER getrs) cannot be stream-captured
        self._bin = torch.zeros((self.NX, self.m), dtype=torch.float64, device=self.device)
        cur = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(cur)
        try:
            with torch.cuda.stream(s):
                self._solve_lines(self._bin)      # warm-up outside the capture (library workspaces)
            cur.wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with no_gc(), torch.cuda.graph(g):
                self._xout = self._solve_lines(self._bin)
            self._graph = g
            return True
        except RuntimeError:
            torch.cuda.synchronize(self.device)
            self._graph = None
            return False

    def solve1(self, b):
        """x = A^-1 b for a one-component operator; b is a length-N vector in the x-major numbering."""
        if not self.factored:
            raise RuntimeError("factor() first")
        if self.ncomp != 1:
            raise ValueError("solve1 needs ncomp=1")
        NX, NY = self.NX, self.NY
        if getattr(self, "_graph", None) is not None:
            self._bin.copy_(b.reshape(NX, NY))
            self._graph.replay()
            return self._xout.reshape(-1).clone()
        return self._solve_lines(b.reshape(NX, NY).clone()).reshape(-1)

    def solve(self, bu, bv):
        """(J^-1 [bu; bv]) split as (xu, xv); bu, bv are length-N vectors in the x-major numbering."""
        if not self.factored:
            raise RuntimeError("factor() first")
        if self.ncomp != 2:
            raise ValueError("solve needs ncomp=2; use solve1")
        NX, NY = self.NX, self.NY
        if getattr(self, "_graph", None) is not None:
            b3 = self._bin.view(NX, 2, NY)
            b3[:, 0, :] = bu.reshape(NX, NY)
            b3[:, 1, :] = bv.reshape(NX, NY)
            self._graph.replay()
            out = self._xout.view(NX, 2, NY)
            return out[:, 0, :].reshape(-1).clone(), out[:, 1, :].reshape(-1).clone()
        B = torch.stack((bu.reshape(NX, NY), bv.reshape(NX, NY)), dim=1).reshape(NX, self.m)
        out = self._solve_lines(B).view(NX, 2, NY)
        return out[:, 0, :].reshape(-1), out[:, 1, :].reshape(-1)
