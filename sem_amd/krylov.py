"""Device-resident GMRES for the solver counterparts.

The reference solves its Newton updates with SciPy's LGMRES on a LinearOperator
(ConvectionDiffusion_Solver.py:123-156, NavierStokes_Solver.py:197-229), with
`inner_m = int(0.3 N)` -- in practice unrestarted GMRES -- and stops when the
residual 2-norm is <= atol = mtol * sqrt(N) (rtol = 0).  Its run time is the
Arnoldi orthogonalisation on the host (12.2 of 15.3 s at 32x32, P=8).

Here the Krylov basis lives in device memory as one (m+1) x N matrix; each
iteration applies the operator (one fused HIP kernel launch) and orthogonalises
with classical Gram-Schmidt done twice (CGS2, as stable as modified Gram-Schmidt),
the second pass's coefficients taken from the basis' Gram matrix: 3 GEMV sweeps over
the basis per iteration (rocBLAS through torch) instead of 4, or 2k BLAS-1 calls for MGS.  Only the (m+1) x m Hessenberg least-squares problem (Givens
rotations) runs on the host.  Vectors are torch tensors on any device, so the
algorithm is unit-tested on CPU against SciPy.
"""
import math

import numpy as np
import torch


class _DeviceSweeps:
    """The two basis passes of an Arnoldi step as HIP kernels (include/sem_ops.h: sem_basis_dot2,
    sem_basis_update): one HBM pass over the basis each, instead of torch's GEMV / skinny-GEMM
    routes.  Used for device tensors without a distributed inner product."""

    def __init__(self, V):
        if V.dtype != torch.float64 or not V.is_cuda or V.stride(1) != 1:
            raise ValueError("the HIP basis sweeps need a float64 device basis with unit column stride")
        from . import _lib
        self.lib = _lib.load()
        self.check = _lib.check
        self.V, self.ldv = V, V.stride(0)
        rows = V.shape[0]
        self.out = torch.empty((rows, 2), dtype=V.dtype, device=V.device)
        self.work = torch.empty(max(1, self.lib.sem_basis_dot2_work_size(rows)), dtype=V.dtype, device=V.device)

    def _stream(self):
        return torch.cuda.current_stream(self.V.device).cuda_stream

    def _vec(self, t, name):
        V = self.V
        if t.dtype != torch.float64 or t.device != V.device or not t.is_contiguous() or t.numel() != V.shape[1]:
            raise ValueError(f"{name} must be a contiguous float64 vector of {V.shape[1]} entries on {V.device}")

    def dot2(self, k, a, b):
        """[V_j . a, V_j . b] for the first k rows -> (k, 2) view."""
        self._vec(a, "a")
        self._vec(b, "b")
        self.check(self.lib.sem_basis_dot2(self.V.data_ptr(), self.ldv, k, self.V.shape[1], a.data_ptr(),
                                           b.data_ptr(), self.work.data_ptr(), self.out.data_ptr(), self._stream()))
        return self.out[:k]

    def update(self, k, c, w):
        """w -= V[:k]^T c, in place."""
        self._vec(w, "w")
        if c.dtype != torch.float64 or c.device != self.V.device or not c.is_contiguous() or c.numel() < k:
            raise ValueError("c must be a contiguous float64 vector of >= k entries on the basis device")
        self.check(self.lib.sem_basis_update(self.V.data_ptr(), self.ldv, k, self.V.shape[1], c.data_ptr(),
                                             w.data_ptr(), self._stream()))


class GMRESResult:
    def __init__(self, x, info, iters, res_norm, matvecs):
        self.x, self.info, self.iters, self.res_norm, self.matvecs = x, info, iters, res_norm, matvecs


def gmres(matvec, b, x0=None, atol=0.0, rtol=0.0, restart=None, maxiter=None, precond=None, callback=None,
          inner=None):
    """Right-preconditioned restarted GMRES.

    matvec(v) -> A v and precond(v) -> M^-1 v take and return 1-D tensors like b.
    Converges when ||b - A x||_2 <= max(atol, rtol * ||b||_2) (SciPy's criterion).
    info = 0 on convergence, else the number of iterations performed (SciPy's convention).
    inner(V, w) -> V @ w (k inner products) replaces the local products; a partitioned solve passes
    sem_amd.parallel.DistributedInner, so every rank sees the same Hessenberg entries and takes the
    same path through the iteration.
    """
    proj = inner if inner is not None else (lambda A, w: A @ w)

    def vnorm(w):
        if inner is None:
            return torch.linalg.vector_norm(w).item()
        return math.sqrt(max(proj(w.unsqueeze(0), w)[0].item(), 0.0))

    N = b.numel()
    dt, dev = b.dtype, b.device
    restart = min(N, restart or 100)
    maxiter = maxiter or 10 * N
    x = torch.zeros_like(b) if x0 is None else x0.clone()
    bnorm = vnorm(b)
    tol = max(atol, rtol * bnorm)
    V = torch.empty((restart + 1, N), dtype=dt, device=dev)
    G = torch.zeros((restart + 1, restart + 1), dtype=dt, device=dev)  # Gram matrix V^T V of the basis
    # the HIP sweeps read and write doubles: other dtypes take torch's GEMV route
    sweeps = _DeviceSweeps(V) if (inner is None and V.is_cuda and V.dtype == torch.float64) else None
    Z = torch.empty((restart, N), dtype=dt, device=dev) if precond is not None else None
    total, matvecs = 0, 0
    r = b - matvec(x) if x0 is not None else b.clone()
    matvecs += x0 is not None
    beta = vnorm(r)
    while True:
        if beta <= tol:
            return GMRESResult(x, 0, total, beta, matvecs)
        if total >= maxiter:
            return GMRESResult(x, total, total, beta, matvecs)
        V[0] = r / beta
        H = np.zeros((restart + 1, restart))
        # Givens rotations and the rotated right-hand side as Python floats: the O(k) rotation
        # sweep per iteration runs in the interpreter, where float arithmetic is several times
        # cheaper than on NumPy scalars (it dominated the host time of long unrestarted solves)
        cs, sn = [0.0] * restart, [0.0] * restart
        g = [0.0] * (restart + 1)
        g[0] = beta
        k_done = 0
        for k in range(restart):
            zk = precond(V[k]) if precond is not None else V[k]
            if Z is not None:
                Z[k] = zk
            w = matvec(zk)
            matvecs += 1
            Vk = V[:k + 1]
            # CGS2 in three sweeps over the basis instead of four: the second pass's coefficients
            # V^T (w - V h) = (I - G) h come from the basis' Gram matrix G = V^T V, whose new row
            # V^T v_k costs one GEMV per iteration.  (One GEMM over [w, v_k] would make it two
            # sweeps, but torch routes that skinny product to a GEMM 14x slower than two GEMVs.)
            if sweeps is not None:           # one HIP pass: CGS pass 1 and the Gram row together
                S = sweeps.dot2(k + 1, w.contiguous(), V[k])
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
            col = hh.cpu().tolist()
            hn = vnorm(w)
            col.append(hn)
            for i in range(k):               # apply previous Givens rotations
                c, s_ = cs[i], sn[i]
                a, b_ = col[i], col[i + 1]
                col[i] = c * a + s_ * b_
                col[i + 1] = -s_ * a + c * b_
            den = math.hypot(col[k], col[k + 1])
            cs[k], sn[k] = (1.0, 0.0) if den == 0.0 else (col[k] / den, col[k + 1] / den)
            col[k] = cs[k] * col[k] + sn[k] * col[k + 1]
            col[k + 1] = 0.0
            H[:k + 2, k] = col
            g[k + 1] = -sn[k] * g[k]
            g[k] = cs[k] * g[k]
            total += 1
            k_done = k + 1
            est = abs(g[k + 1])
            if callback is not None:
                callback(est)
            if est <= tol or hn == 0.0 or total >= maxiter:
                break
            V[k + 1] = w / hn
        # x += Z y  with  H[:k,:k] y = g[:k]
        y = np.linalg.solve(np.triu(H[:k_done, :k_done]), np.asarray(g[:k_done])) if k_done else np.zeros(0)
        yt = torch.as_tensor(y, dtype=dt, device=dev)
        basis = Z[:k_done] if Z is not None else V[:k_done]
        x = x + basis.T @ yt
        r = b - matvec(x)
        matvecs += 1
        beta = vnorm(r)


def gmres_left(matvec, b, x0=None, atol=0.0, rtol=0.0, restart=20, maxiter=None, precond=None, callback=None):
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
    """
    N = b.numel()
    dt, dev = b.dtype, b.device
    restart = min(N, restart or 20)
    maxiter = maxiter or 10 * N
    psolve = precond if precond is not None else (lambda t: t)
    x = torch.zeros_like(b) if x0 is None else x0.clone()
    bnorm = torch.linalg.vector_norm(b).item()
    if bnorm == 0.0:
        return GMRESResult(torch.zeros_like(b), 0, 0, 0.0, 0)
    tol = max(atol, rtol * bnorm)
    eps = np.finfo(np.float64).eps
    ptol_max = 1.0
    ptol = torch.linalg.vector_norm(psolve(b)).item() * min(ptol_max, tol / bnorm)
    V = torch.empty((restart + 1, N), dtype=dt, device=dev)
    total, matvecs = 0, 0
    r = b - matvec(x) if x0 is not None else b.clone()
    matvecs += x0 is not None
    rnorm = torch.linalg.vector_norm(r).item()
    if rnorm < tol:
        return GMRESResult(x, 0, 0, rnorm, matvecs)
    for _ in range(maxiter):
        z = psolve(r)
        zn = torch.linalg.vector_norm(z).item()
        V[0] = z / zn
        H = np.zeros((restart + 1, restart))
        cs, sn = np.zeros(restart), np.zeros(restart)
        g = np.zeros(restart + 1)
        g[0] = zn
        breakdown, presid, k_done = False, 0.0, 0
        for k in range(restart):
            w = psolve(matvec(V[k]))
            matvecs += 1
            h0 = torch.linalg.vector_norm(w).item()
            Vk = V[:k + 1]
            h = Vk @ w                       # CGS2 in place of SciPy's MGS
            w = w - Vk.T @ h
            h2 = Vk @ w
            w = w - Vk.T @ h2
            H[:k + 1, k] = (h + h2).cpu().numpy()
            hn = torch.linalg.vector_norm(w).item()
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
        rnorm = torch.linalg.vector_norm(r).item()
        if rnorm <= tol or breakdown:
            break
        if presid <= ptol:
            ptol_max = max(eps, 0.25 * ptol_max)
        else:
            ptol_max = min(1.0, 1.5 * ptol_max)
        ptol = presid * min(ptol_max, tol / rnorm)
    return GMRESResult(x, 0 if rnorm <= tol else maxiter, total, rnorm, matvecs)
