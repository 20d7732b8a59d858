"""Device-resident GMRES for the solver counterparts.

The reference solves its Newton updates with SciPy's LGMRES on a LinearOperator
(ConvectionDiffusion_Solver.py:123-156, NavierStokes_Solver.py:197-229), with
`inner_m = int(0.3 N)` -- in practice unrestarted GMRES -- and stops when the
residual 2-norm is <= atol = mtol * sqrt(N) (rtol = 0).  Its run time is the
Arnoldi orthogonalisation on the host (12.2 of 15.3 s at 32x32, P=8).

Here the Krylov basis lives in device memory as one (m+1) x N matrix; each
iteration applies the operator (one fused HIP kernel launch) and orthogonalises
with classical Gram-Schmidt done twice (CGS2), the second pass's coefficients taken from the
basis' Gram matrix: (I - G) h equals V^T (w - V h) in exact arithmetic, so two sweeps over the
basis per iteration instead of four (the HIP kernels sem_basis_dot2 / sem_basis_update).  That form
cannot see the rounding error of the first subtraction, so when ||w|| collapses by more than
REORTH_ETA = 1e-4 (severe cancellation, where the loss of orthogonality eps ||w|| / h_{k+1,k} would
exceed ~1e-12) a true extra pass is made; tests/test_krylov.py checks ||I - V^T V|| on an
ill-conditioned system.  Only the (m+1) x m Hessenberg least-squares problem (Givens
rotations) runs on the host.  Vectors are torch tensors on any device, so the
algorithm is unit-tested on CPU against SciPy.
"""
import math
import os

import numpy as np
import torch

from . import tracing
from .tracing import phase


class _DeviceSweeps:
    """The two basis passes of an Arnoldi step as HIP kernels (include/sem_ops.h: sem_basis_dot2,
    sem_basis_update): one HBM pass over the basis each, instead of torch's GEMV / skinny-GEMM
    routes.  `segments`: the entries this rank owns (a partitioned vector's shared interface line is
    counted on one rank only); dot2 runs over those ranges -- pointer offsets into V, a and b, no mask
    -- and the update over the whole local vector."""

    def __init__(self, V, segments=None):
        if V.dtype != torch.float64 or not V.is_cuda or V.stride(1) != 1:
            raise ValueError("the HIP basis sweeps need a float64 device basis with unit column stride")
        from . import _lib
        self.lib = _lib.load()
        self.check = _lib.check
        self.V, self.ldv = V, V.stride(0)
        n = V.shape[1]
        self.segments = [(0, n)] if segments is None else [(int(a), int(b)) for a, b in segments if b > a]
        rows = V.shape[0]
        self.out = torch.empty((len(self.segments), rows, 2), dtype=V.dtype, device=V.device)
        self.work = torch.empty(max(1, max(self.lib.sem_basis_dot2_work_size(rows, b - a) for a, b in self.segments)
                                    if self.segments else 1), dtype=V.dtype, device=V.device)

    def _stream(self):
        return torch.cuda.current_stream(self.V.device).cuda_stream

    def _vec(self, t, name):
        V = self.V
        if t.dtype != torch.float64 or t.device != V.device or not t.is_contiguous() or t.numel() != V.shape[1]:
            raise ValueError(f"{name} must be a contiguous float64 vector of {V.shape[1]} entries on {V.device}")

    def dot2(self, k, a, b):
        """[V_j . a, V_j . b] over the owned entries for the first k rows -> (k, 2)."""
        self._vec(a, "a")
        self._vec(b, "b")
        if not self.segments:
            return torch.zeros((k, 2), dtype=self.V.dtype, device=self.V.device)
        V, s = self.V, self._stream()
        for i, (lo, hi) in enumerate(self.segments):
            off = lo * V.element_size()
            self.check(self.lib.sem_basis_dot2(V.data_ptr() + off, self.ldv, k, hi - lo, a.data_ptr() + off,
                                               b.data_ptr() + off, self.work.data_ptr(), self.out[i].data_ptr(), s))
        return self.out[0, :k] if len(self.segments) == 1 else self.out[:, :k].sum(0)

    def sqnorm(self, w):
        """w . w over the owned entries (0-d device tensor)."""
        return _seg_sqnorm(w, self.segments)

    def update(self, k, c, w):
        """w -= V[:k]^T c, in place."""
        self._vec(w, "w")
        if c.dtype != torch.float64 or c.device != self.V.device or not c.is_contiguous() or c.numel() < k:
            raise ValueError("c must be a contiguous float64 vector of >= k entries on the basis device")
        self.check(self.lib.sem_basis_update(self.V.data_ptr(), self.ldv, k, self.V.shape[1], c.data_ptr(),
                                             w.data_ptr(), self._stream()))


def _seg_sqnorm(w, segments):
    s = None
    for a, b in segments:
        p = torch.dot(w[a:b], w[a:b])
        s = p if s is None else s + p
    return s if s is not None else torch.zeros((), dtype=w.dtype, device=w.device)


class _TorchSweeps:
    """The same two passes through torch (CPU tensors, other dtypes): the CPU tests run the algorithm the
    device runs, partitioned or not."""

    def __init__(self, V, segments=None):
        self.V = V
        n = V.shape[1]
        self.segments = [(0, n)] if segments is None else [(int(a), int(b)) for a, b in segments if b > a]

    def dot2(self, k, a, b):
        V = self.V
        out = torch.zeros((k, 2), dtype=V.dtype, device=V.device)
        for lo, hi in self.segments:
            out += torch.stack((V[:k, lo:hi] @ a[lo:hi], V[:k, lo:hi] @ b[lo:hi]), dim=1)
        return out

    def update(self, k, c, w):
        w -= self.V[:k].T @ c[:k]

    def sqnorm(self, w):
        return _seg_sqnorm(w, self.segments)


REORTH_ETA = 1e-4   # a true extra orthogonalisation pass when ||w|| drops below this fraction


class GMRESResult:
    """matvecs counts the operator applications the iteration used; `discarded` the speculative ones of the
    pipelined step that were thrown away (on convergence or after a reorthogonalisation)."""

    def __init__(self, x, info, iters, res_norm, matvecs, reorth=0, discarded=0):
        self.x, self.info, self.iters, self.res_norm, self.matvecs = x, info, iters, res_norm, matvecs
        self.reorth, self.discarded = reorth, discarded


def _sizes(N, restart, maxiter, inner, default_restart):
    """Restart length and iteration cap.  A partitioned solve (inner given) sizes nothing from its local
    length N: ranks holding strips of different sizes would otherwise leave the Arnoldi loop at different
    iterations and their collectives would mismatch (found by the world-8 gloo test of the NS update with
    one-column strips); the caller passes sizes every rank shares."""
    if inner is not None:
        if maxiter is None:
            raise ValueError("a partitioned Krylov solve needs maxiter (a size every rank shares)")
        return restart or default_restart, maxiter
    return min(N, restart or default_restart), maxiter or 10 * N


def _host64(t):
    """A 1-D tensor as a contiguous float64 NumPy array on the host."""
    return np.ascontiguousarray(t.detach().cpu().numpy(), dtype=np.float64)


_GIVENS = []


def givens_column(col, cs, sn, g, k):
    """One GMRES least-squares column: rotations 0..k-1 (cs, sn) applied to col[0..k+1], rotation k formed from
    (col[k], col[k+1]) and applied to col and to g[k], g[k+1] -- in C (sem_givens_column, the library's host
    code) when the library loads, else the same loop in Python.  float64 arrays, updated in place."""
    if not _GIVENS:
        try:
            from . import _lib
            _GIVENS.append(_lib.load())
        except (OSError, RuntimeError, ImportError):
            _GIVENS.append(None)
    lib = _GIVENS[0]
    if lib is not None:
        from . import _lib
        _lib.check(lib.sem_givens_column(col.ctypes.data, cs.ctypes.data, sn.ctypes.data, g.ctypes.data, int(k)))
        return
    for i in range(k):
        c, s_ = cs[i], sn[i]
        a, b_ = col[i], col[i + 1]
        col[i] = c * a + s_ * b_
        col[i + 1] = -s_ * a + c * b_
    den = math.hypot(col[k], col[k + 1])
    cs[k], sn[k] = (1.0, 0.0) if den == 0.0 else (col[k] / den, col[k + 1] / den)
    col[k] = cs[k] * col[k] + sn[k] * col[k + 1]
    col[k + 1] = 0.0
    g[k + 1] = -sn[k] * g[k]
    g[k] = cs[k] * g[k]


def gmres(matvec, b, x0=None, atol=0.0, rtol=0.0, restart=None, maxiter=None, precond=None, callback=None,
          inner=None, basis_out=None, linear_precond=True):
    """Right-preconditioned restarted GMRES.

    matvec(v) -> A v and precond(v) -> M^-1 v take and return 1-D tensors like b.
    Converges when ||b - A x||_2 <= max(atol, rtol * ||b||_2) (SciPy's criterion).
    info = 0 on convergence, else the number of iterations performed (SciPy's convention).
    inner: the inner product of a partitioned vector.  sem_amd.parallel.DistributedInner (owned `segments` of
    the local vector and a `reduce` all-reduce) keeps the partitioned solve on the HIP basis sweeps: per Arnoldi
    step one all-reduce of both CGS2 coefficient sets with ||w||^2, one of ||w||^2 after the update, and the
    pipelined step as on one GPU -- every rank sees the same Hessenberg entries and takes the same path through
    the iteration.  Any other callable inner(V, w) -> V @ w takes torch's route (one collective per product).
    basis_out: a list that receives a copy of each cycle's orthonormal basis (tests).
    linear_precond: precond is a fixed linear map (the solvers' mass diagonal, PCD and direct solves), so the
    correction is M^-1 (V y) and the preconditioned basis Z = M^-1 V is not kept -- half the basis memory, and
    twice the vectors within a memory budget; False keeps Z (flexible GMRES, for a varying preconditioner).
    """
    N = b.numel()
    dt, dev = b.dtype, b.device
    restart, maxiter = _sizes(N, restart, maxiter, inner, 100)
    segments = getattr(inner, "segments", None) if inner is not None else None
    red = getattr(inner, "reduce", None) if segments is not None else None
    generic = inner is not None and segments is None      # an arbitrary inner(V, w) callable
    proj = inner
    x = torch.zeros_like(b) if x0 is None else x0.clone()
    V = torch.empty((restart + 1, N), dtype=dt, device=dev)
    G = torch.zeros((restart + 1, restart + 1), dtype=dt, device=dev)  # Gram matrix V^T V of the basis
    sweeps = None
    if not generic:   # the HIP sweeps read and write doubles: CPU tensors and other dtypes take torch's
        sweeps = (_DeviceSweeps(V, segments) if (V.is_cuda and V.dtype == torch.float64)
                  else _TorchSweeps(V, segments))

    def dnorm(w):
        """||w|| over every rank as a 0-d device tensor (no host synchronisation)."""
        if red is None:
            return torch.linalg.vector_norm(w)
        return torch.sqrt(red(sweeps.sqnorm(w).reshape(1))[0].clamp_min(0.0))

    def vnorm(w):
        if generic:
            return math.sqrt(max(proj(w.unsqueeze(0), w)[0].item(), 0.0))
        return float(dnorm(w))

    bnorm = vnorm(b)
    tol = max(atol, rtol * bnorm)
    Z = torch.empty((restart, N), dtype=dt, device=dev) if (precond is not None and not linear_precond) else None
    total, matvecs, discarded = 0, 0, 0
    self_reorth = [0]
    # pipelined steps on the GPU, partitioned or not (SEM_GMRES_PIPELINE=0 turns them off; cfg4's Ra = 1e6 block
    # solve 0.744 -> 0.715 s, profiles/r04/schur_ab/schurpipe_*.jsonl): a pinned host buffer for each step's
    # coefficients and norms, and the event that marks its copy
    pipe = None
    # a host-staged reduce (gloo rehearsals of the partitioned solve) synchronises the host with the device at every
    # collective, the matvec's own included: nothing can run behind the host's wait, so no speculation there
    bdev = getattr(inner, "bdev", None) if red is not None else None
    staged = bdev is not None and bdev.type != dev.type
    if isinstance(sweeps, _DeviceSweeps) and not staged and os.environ.get("SEM_GMRES_PIPELINE", "1") != "0":
        pipe = (torch.empty(restart + 3, dtype=torch.float64, pin_memory=True), torch.cuda.Event())
    r = b - matvec(x) if x0 is not None else b.clone()
    matvecs += x0 is not None
    beta = vnorm(r)
    while True:
        if beta <= tol:
            return GMRESResult(x, 0, total, beta, matvecs, self_reorth[0], discarded)
        if total >= maxiter:
            return GMRESResult(x, total, total, beta, matvecs, self_reorth[0], discarded)
        V[0] = r / beta
        H = np.zeros((restart + 1, restart))
        # Givens rotations and the rotated right-hand side in float64 arrays: the O(k) rotation sweep of
        # each step runs in C (sem_givens_column), not in the interpreter (~0.6 us per earlier rotation there:
        # ~1 ms per step at k ~ 1,600, with the GPU idle behind the step's host synchronisation)
        cs, sn = np.zeros(restart), np.zeros(restart)
        g = np.zeros(restart + 1)
        g[0] = beta
        k_done = 0
        pending = None   # the next step's A M^-1 v_{k+1}, launched before this step's host synchronisation
        for k in range(restart):
            if pending is None:
                with phase("krylov.matvec"):
                    zk = precond(V[k]) if precond is not None else V[k]
                    if Z is not None:
                        Z[k] = zk
                    w = matvec(zk)
                matvecs += 1
            else:
                w, pending = pending, None
            w_in = w
            Vk = V[:k + 1]
            tok = tracing.begin("krylov.orthogonalise")
            # CGS2 in three sweeps over the basis instead of four: the second pass's coefficients
            # V^T (w - V h) = (I - G) h come from the basis' Gram matrix G = V^T V, whose new row
            # V^T v_k costs one GEMV per iteration.  (One GEMM over [w, v_k] would make it two
            # sweeps, but torch routes that skinny product to a GEMM 14x slower than two GEMVs.)
            h0sq = None
            if sweeps is not None:           # one pass: CGS pass 1 and the Gram row together
                w = w.contiguous()
                S = sweeps.dot2(k + 1, w, V[k])
                if red is not None:          # ONE all-reduce: both coefficient sets and ||w||^2
                    buf = torch.cat((S.reshape(-1), sweeps.sqnorm(w).reshape(1)))
                    red(buf)
                    h, gk, h0sq = buf[0:2 * k + 2:2], buf[1:2 * k + 2:2], buf[-1]
                else:
                    h, gk = S[:, 0].clone(), S[:, 1].clone()
            else:
                h = proj(Vk, w)              # CGS pass 1
                gk = proj(Vk, V[k])          # Gram row of the newest basis vector
            G[k, :k + 1] = gk
            G[:k + 1, k] = gk
            hh = 2.0 * h - G[:k + 1, :k + 1] @ h   # h + (I - G) h: both passes' coefficients
            if sweeps is not None:
                w = w.clone()
                sweeps.update(k + 1, hh.contiguous(), w)
            else:
                w = w - Vk.T @ hh
            spec = None
            if sweeps is not None:
                nw = dnorm(w)
                n0 = torch.linalg.vector_norm(w_in) if h0sq is None else torch.sqrt(h0sq.clamp_min(0.0))
                pk = torch.cat((hh, nw[None], n0[None]))
            tracing.end(tok)
            if pipe is not None:
                # pipelined step: the coefficients and norms go to pinned host memory, then v_{k+1} = w / ||w|| and
                # the next matvec are queued BEFORE the host waits for that copy, so the GPU runs the next operator
                # application while the host does this step's least-squares update; the speculation is dropped on
                # convergence and redone after a reorthogonalisation (which changes w).  A zero ||w|| (exact
                # breakdown) divides by one instead: the speculation is dropped there anyway.
                pipe[0][:k + 3].copy_(pk, non_blocking=True)
                pipe[1].record()
                if k + 1 < restart and total + 1 < maxiter:
                    with phase("krylov.matvec"):
                        V[k + 1] = w / torch.where(nw > 0, nw, torch.ones_like(nw))
                        z1 = precond(V[k + 1]) if precond is not None else V[k + 1]
                        if Z is not None:
                            Z[k + 1] = z1
                        spec = matvec(z1)
                    matvecs += 1
                with phase("krylov.host_wait"):
                    pipe[1].synchronize()
                cn = pipe[0][:k + 3].numpy().copy()
            elif sweeps is not None:   # one device -> host transfer per step: coefficients, ||w|| after and before
                with phase("krylov.host_wait"):
                    cn = _host64(pk)
            if sweeps is not None:
                h0 = float(cn[-1])
                col = cn[:-1]
                hn = float(col[-1])
            else:
                col = np.empty(k + 2)
                col[:k + 1] = _host64(hh)
                hn = vnorm(w)
                h0 = vnorm(w_in)
                col[k + 1] = hn
            if hn < REORTH_ETA * h0:
                # severe cancellation: the Gram-matrix form of the second pass cannot see the rounding
                # error of the first subtraction, so make one true extra pass (it fires only when
                # ||w|| collapses by 1e4 or more)
                if sweeps is not None:
                    h2 = sweeps.dot2(k + 1, w, V[k])[:, 0].clone()
                    if red is not None:
                        red(h2)
                    sweeps.update(k + 1, h2.contiguous(), w)
                else:
                    h2 = proj(Vk, w)
                    w = w - Vk.T @ h2
                hn = vnorm(w)
                col[:k + 1] += _host64(h2)
                col[k + 1] = hn
                self_reorth[0] += 1
                if spec is not None:   # v_{k+1} and the speculative matvec came from the unreorthogonalised w
                    spec, matvecs, discarded = None, matvecs - 1, discarded + 1
            givens_column(col, cs, sn, g, k)   # earlier rotations, the new one, the right-hand side
            H[:k + 2, k] = col
            total += 1
            k_done = k + 1
            est = abs(float(g[k + 1]))
            if callback is not None:
                callback(est)
            if est <= tol or hn == 0.0 or total >= maxiter:
                if spec is not None:   # the speculation past convergence is not used
                    matvecs, discarded = matvecs - 1, discarded + 1
                break
            if spec is not None:
                pending = spec    # V[k+1] and A M^-1 V[k+1] (and Z[k+1]) are already on the device
            else:
                V[k + 1] = w / hn
        if basis_out is not None:
            basis_out.append(V[:k_done].clone())
        # x += Z y (= M^-1 V y for a linear preconditioner)  with  H[:k,:k] y = g[:k]
        y = np.linalg.solve(np.triu(H[:k_done, :k_done]), np.asarray(g[:k_done])) if k_done else np.zeros(0)
        yt = torch.as_tensor(y, dtype=dt, device=dev)
        if Z is not None:
            x = x + Z[:k_done].T @ yt
        elif precond is not None:
            x = x + precond(V[:k_done].T @ yt)
        else:
            x = x + V[:k_done].T @ yt
        r = b - matvec(x)
        matvecs += 1
        beta = vnorm(r)


def gmres_left(matvec, b, x0=None, atol=0.0, rtol=0.0, restart=20, maxiter=None, precond=None, callback=None,
               inner=None, jump=None, jump_ratio=10.0):
    """Left-preconditioned restarted GMRES, SciPy's `gmres` (scipy 1.15 iterative.py) restated on
    device tensors: the Arnoldi process runs on M^-1 A, the inner loop stops on the
    preconditioned residual estimate against an adaptive tolerance (gh-8400 control), and each
    restart checks the true residual ||b - A x||_2 <= max(atol, rtol ||b||_2).

    The Boussinesq coupler needs this variant (OpenMDAO's ScipyKrylov hands its block-Jacobi
    preconditioner to SciPy as M): M^-1 is only ever applied to b, to residuals b - A x and to
    products A v -- vectors in the range of A.  The NS block solve (a Schur complement with
    spurious pressure modes of the equal-order P_N-P_N discretisation) needs its right-hand side
    in that range; the Arnoldi vectors a right-preconditioned GMRES feeds M^-1 are not.
    `maxiter` counts restarts, as SciPy's does.  info = 0 on convergence, else maxiter.
    inner(A, w) = A @ w over a partitioned vector (sem_amd.parallel: shared lines counted once, the
    partial products all-reduced); norms follow it.

    jump (round 6): safeguard for an INEXACT preconditioner.  With a fixed M, the preconditioned
    residual ||M^-1 (b - A x)|| that starts a cycle equals the estimate the previous cycle ended with; the coupler's
    M^-1 is a pair of iterative block solves stopped at an absolute tolerance, i.e. a slightly different operator at
    every application, and when that inconsistency builds up the restart finds a true residual far above the
    estimate (cfg5, Ra = 1e4: 20x and then 280x before the Newton iteration diverged, profiles/r05/cfg5/).  When the
    new cycle's residual exceeds jump_ratio times the last estimate, jump(ratio) is called; if it returns True (the
    caller tightened its preconditioner) the cycle's first vector is recomputed with the tightened M.  The outer
    arithmetic is SciPy's either way; result.jumps counts the detections."""
    N = b.numel()
    dt, dev = b.dtype, b.device
    restart, maxiter = _sizes(N, restart, maxiter, inner, 20)
    psolve = precond if precond is not None else (lambda t: t)
    if inner is None:
        dot = lambda A, w: A @ w  # noqa: E731
        vnorm = lambda t: torch.linalg.vector_norm(t).item()  # noqa: E731
    else:
        dot = inner
        vnorm = lambda t: math.sqrt(max(float(inner(t[None], t)[0]), 0.0))  # noqa: E731
    x = torch.zeros_like(b) if x0 is None else x0.clone()
    bnorm = vnorm(b)
    if bnorm == 0.0:
        return GMRESResult(torch.zeros_like(b), 0, 0, 0.0, 0)
    tol = max(atol, rtol * bnorm)
    eps = np.finfo(np.float64).eps
    ptol_max = 1.0
    ptol = vnorm(psolve(b)) * min(ptol_max, tol / bnorm)
    V = torch.empty((restart + 1, N), dtype=dt, device=dev)
    total, matvecs = 0, 0
    r = b - matvec(x) if x0 is not None else b.clone()
    matvecs += x0 is not None
    rnorm = vnorm(r)
    if rnorm < tol:
        return GMRESResult(x, 0, 0, rnorm, matvecs)
    jumps, prev_presid = 0, None
    for _ in range(maxiter):
        z = psolve(r)
        zn = vnorm(z)
        if jump is not None and prev_presid and zn > jump_ratio * prev_presid:
            jumps += 1
            if jump(zn / prev_presid):
                z = psolve(r)
                zn = vnorm(z)
        V[0] = z / zn
        H = np.zeros((restart + 1, restart))
        cs, sn = np.zeros(restart), np.zeros(restart)
        g = np.zeros(restart + 1)
        g[0] = zn
        breakdown, presid, k_done = False, 0.0, 0
        for k in range(restart):
            w = psolve(matvec(V[k]))
            matvecs += 1
            h0 = vnorm(w)
            Vk = V[:k + 1]
            h = dot(Vk, w)                   # CGS2 in place of SciPy's MGS
            w = w - Vk.T @ h
            h2 = dot(Vk, w)
            w = w - Vk.T @ h2
            H[:k + 1, k] = (h + h2).cpu().numpy()
            hn = vnorm(w)
            if hn <= eps * h0:               # exact-solution indicator
                H[k + 1, k], breakdown = 0.0, True
            else:
                H[k + 1, k] = hn
                V[k + 1] = w / hn
            for i in range(k):
                t = cs[i] * H[i, k] + sn[i] * H[i + 1, k]
                H[i + 1, k] = -sn[i] * H[i, k] + cs[i] * H[i + 1, k]
                H[i, k] = t
            den = math.hypot(H[k, k], H[k + 1, k])
            cs[k], sn[k] = (1.0, 0.0) if den == 0.0 else (H[k, k] / den, H[k + 1, k] / den)
            H[k, k], H[k + 1, k] = den, 0.0
            g[k + 1] = -sn[k] * g[k]
            g[k] = cs[k] * g[k]
            presid = abs(g[k + 1])
            total += 1
            k_done = k + 1
            if callback is not None:
                callback(presid)
            if presid <= ptol or breakdown:
                break
        Hk = np.triu(H[:k_done, :k_done]).copy()
        gk = g[:k_done].copy()
        if Hk[-1, -1] == 0.0:
            gk[-1], Hk[-1, -1] = 0.0, 1.0
        y = np.linalg.solve(Hk, gk)
        x = x + V[:k_done].T @ torch.as_tensor(y, dtype=dt, device=dev)
        r = b - matvec(x)
        matvecs += 1
        rnorm = vnorm(r)
        if rnorm <= tol or breakdown:
            break
        prev_presid = presid
        if presid <= ptol:
            ptol_max = max(eps, 0.25 * ptol_max)
        else:
            ptol_max = min(1.0, 1.5 * ptol_max)
        ptol = presid * min(ptol_max, tol / rnorm)
    res = GMRESResult(x, 0 if rnorm <= tol else maxiter, total, rnorm, matvecs)
    res.jumps = jumps
    return res


class Recycle:
    """Recycled Krylov subspace for a sequence of solves with ONE operator (GCRO, de Sturler 1999).

    Holds U, C with A U = C and C^T C = I.  A solve first takes the part of b in span(C)
    (x0 = U C^T b), keeps its Arnoldi vectors orthogonal to C, and afterwards appends its own search
    space, so every later solve with the same operator starts where the previous ones ended.  The
    coupled Newton-Krylov of the Boussinesq coupler applies each solver's block solve once per
    outer GMRES iteration with a fixed linearisation -- tens of solves per operator.  The solver
    resets it whenever its operator changes.  Device memory: 2 x capacity vectors."""

    def __init__(self, n, dtype, device, capacity):
        self.n, self.cap = n, int(capacity)
        self.buf = torch.empty((self.cap, n), dtype=dtype, device=device)   # C rows, then a cycle's basis
        self.U = torch.empty((self.cap, n), dtype=dtype, device=device)
        self.k = 0
        self.solves = 0
        self.pending = None
        # singular values kept when a cycle joins the space: U = (Z - U E) W S^-1 grows like 1 / s_min,
        # and the rounding error of the projection x0 = U C^T b with it
        self.rcond = 1e-4
        self.first_iters = None   # iterations of the first solve after a reset (stagnation guard)

    def reset(self):
        self.k = 0
        self.pending = None
        self.first_iters = None

    def absorb(self):
        """Append the last cycle's search space (deferred until the space is used again, so a lone
        solve pays nothing): A (Z_m - U E) = V_{m+1} H_m."""
        if self.pending is None:
            return
        kc, m, Zm, E, H0 = self.pending
        self.pending = None
        dt, dev = self.buf.dtype, self.buf.device
        # H_m = P S W^T (thin SVD); directions with tiny singular values (the operator's near-null space,
        # e.g. the spurious pressure modes of the NS Schur complement) are left out, so U stays bounded:
        # A (Z_m - U E) W_r S_r^-1 = V_{m+1} P_r
        P, S, Wt = torch.linalg.svd(torch.as_tensor(H0[:m + 1, :m], dtype=dt, device=dev), full_matrices=False)
        keep = int((S > S[0] * self.rcond).sum().item())
        if keep == 0:
            return
        Cn = P[:, :keep].T @ self.buf[kc:kc + m + 1]
        Un = Zm - (E[:, :m].T @ self.U[:kc] if kc else 0.0)
        Un = (Wt[:keep] / S[:keep, None]) @ Un
        self.buf[kc:kc + keep] = Cn
        self.U[kc:kc + keep] = Un
        self.k = kc + keep


def gcro(matvec, b, x0=None, atol=0.0, rtol=0.0, restart=None, maxiter=None, precond=None, callback=None,
         recycle=None):
    """GMRES with a recycled subspace (GCRO): same stopping rule and result contract as `gmres`
    (||b - A x||_2 <= max(atol, rtol ||b||_2), info = 0 on convergence); right-preconditioned.
    CGS2 as in `gmres`, over the combined basis [C; V]: one dot2 and one update sweep per step."""
    if recycle is None:
        return gmres(matvec, b, x0=x0, atol=atol, rtol=rtol, restart=restart, maxiter=maxiter, precond=precond,
                     callback=callback)
    N = b.numel()
    dt, dev = b.dtype, b.device
    restart = min(N, restart or 100)
    maxiter = maxiter or 10 * N
    vnorm = lambda t: torch.linalg.vector_norm(t).item()  # noqa: E731
    x = torch.zeros_like(b) if x0 is None else x0.clone()
    bnorm = vnorm(b)
    tol = max(atol, rtol * bnorm)
    rc = recycle
    total, matvecs = 0, 0
    r = b - matvec(x) if x0 is not None else b.clone()
    matvecs += x0 is not None

    def project(x, r):
        if rc.k:
            c = rc.buf[:rc.k] @ r
            x = x + rc.U[:rc.k].T @ c
            r = r - rc.buf[:rc.k].T @ c
        return x, r

    rc.absorb()
    x, r = project(x, r)
    beta = vnorm(r)
    sweeps = _DeviceSweeps(rc.buf) if (rc.buf.is_cuda and dt == torch.float64) else None
    while True:
        if beta <= tol:
            rc.solves += 1
            if rc.first_iters is None:
                rc.first_iters = total
            return GMRESResult(x, 0, total, beta, matvecs)
        if total >= maxiter:
            return GMRESResult(x, total, total, beta, matvecs)
        if rc.k and rc.first_iters is not None and total > 2 * rc.first_iters + restart:
            # stagnation (the recycled space limits the attainable accuracy): continue as plain GMRES
            rc.reset()
            rc.first_iters = 0
        if rc.pending is not None:                    # restart: the finished cycle joins C first
            rc.absorb()
            x, r = project(x, r)
            beta = vnorm(r)
        if rc.cap - rc.k - 1 < min(restart, 32):      # full: start a new recycle space
            rc.reset()
        kc = rc.k
        m_max = min(restart, rc.cap - kc - 1)
        full = rc.buf
        V = full[kc:kc + m_max + 1]
        Z = torch.empty((m_max, N), dtype=dt, device=dev) if precond is not None else None
        Gr = torch.zeros((m_max + 1, kc + m_max + 1), dtype=dt, device=dev)   # Gram rows of the V vectors
        E = torch.zeros((kc, m_max), dtype=dt, device=dev)                     # C^T A z_j
        H0 = np.zeros((m_max + 1, m_max))                                      # Hessenberg (unrotated)
        V[0] = r / beta
        cs, sn = [0.0] * m_max, [0.0] * m_max
        g = [0.0] * (m_max + 1)
        g[0] = beta
        Hr = np.zeros((m_max + 1, m_max))
        m = 0
        for j in range(m_max):
            zj = precond(V[j]) if precond is not None else V[j]
            if Z is not None:
                Z[j] = zj
            w = matvec(zj)
            matvecs += 1
            nb = kc + j + 1
            if sweeps is not None:
                S = sweeps.dot2(nb, w.contiguous(), V[j])
                h, gr = S[:, 0].clone(), S[:, 1].clone()
            else:
                h, gr = full[:nb] @ w, full[:nb] @ V[j]
            Gr[j, :nb] = gr
            Gr[:j, kc + j] = gr[kc:kc + j]          # G_VV is symmetric: fill the new column too
            # (G h) with G_CC = I and the V rows' Gram rows Gr: both CGS passes' coefficients
            hC, hV = h[:kc], h[kc:]
            GV = Gr[:j + 1, :nb]
            Gh_C = hC + GV[:, :kc].T @ hV
            Gh_V = GV @ h
            hh = torch.cat((2.0 * hC - Gh_C, 2.0 * hV - Gh_V))
            w = w.clone()
            if sweeps is not None:
                sweeps.update(nb, hh.contiguous(), w)
            else:
                w = w - full[:nb].T @ hh
            E[:, j] = hh[:kc]
            col = torch.cat((hh[kc:], torch.linalg.vector_norm(w)[None])).cpu().tolist()
            hn = col[-1]
            H0[:j + 2, j] = col
            for i in range(j):
                c_, s_ = cs[i], sn[i]
                a, b_ = col[i], col[i + 1]
                col[i] = c_ * a + s_ * b_
                col[i + 1] = -s_ * a + c_ * b_
            den = math.hypot(col[j], col[j + 1])
            cs[j], sn[j] = (1.0, 0.0) if den == 0.0 else (col[j] / den, col[j + 1] / den)
            col[j] = cs[j] * col[j] + sn[j] * col[j + 1]
            col[j + 1] = 0.0
            Hr[:j + 2, j] = col
            g[j + 1] = -sn[j] * g[j]
            g[j] = cs[j] * g[j]
            total += 1
            m = j + 1
            est = abs(g[j + 1])
            if callback is not None:
                callback(est)
            if hn != 0.0:
                V[j + 1] = w / hn      # also on the last step: the recycle update uses V_{m+1}
            if est <= tol or hn == 0.0 or total >= maxiter:
                break
        y = np.linalg.solve(np.triu(Hr[:m, :m]), np.asarray(g[:m]))
        yt = torch.as_tensor(y, dtype=dt, device=dev)
        Zm = Z[:m] if Z is not None else V[:m]
        Ey = E[:, :m] @ yt
        x = x + Zm.T @ yt - (rc.U[:kc].T @ Ey if kc else 0.0)
        if hn != 0.0 and m > 0:      # this cycle's search space joins the recycle space (deferred)
            rc.pending = (kc, m, Zm, E, H0)
        r = b - matvec(x)
        matvecs += 1
        x, r = project(x, r)
        beta = vnorm(r)
