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
import os
import time

import torch

from ..device import no_gc

GEMV_LDS_DOUBLES = 8192   # sem_block_gemv stages S m operand doubles in LDS (include/sem_ops.h)


def _inverse(A):
    """torch.linalg.inv of a batch; on a getrf workspace-allocation failure the batch is halved."""
    try:
        return torch.linalg.inv(A)
    except RuntimeError as e:
        if "ALLOC_FAILED" not in str(e) or A.dim() < 3 or A.shape[0] == 1:
            raise
    out = torch.empty_like(A)
    step = max(1, A.shape[0] // 2)
    for i in range(0, A.shape[0], step):
        out[i:i + step] = _inverse(A[i:i + step])
    return out


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


def batched_inverse(A, max_batch=128):
    """Inverses of a batch of blocks (rocSOLVER getrf/getri through torch), checked.

    Measured on MI355X (tools/chunk_probe.py, profiles/r02/cfg5/chunk_probe.txt): the batched
    inverse returns wrong blocks, without an error, for some shapes -- 121^2 blocks (the one-component
    element interiors at P = 12) in batches of 384 and more -- and has been seen to fail its workspace
    allocation for others (64 blocks of 455^2).  So the batch is inverted in slices of max_batch blocks,
    every block is checked through its residual A X - I, and a block that misses is inverted again on
    its own (then by a solve against the identity) before giving up."""
    if A.dim() < 3:
        return torch.linalg.inv(A)
    out = torch.empty_like(A)
    for i in range(0, A.shape[0], max_batch):
        a = A[i:i + max_batch]
        x = _inverse(a)
        for j in _bad_blocks(a, x).tolist():
            xj = torch.linalg.inv(a[j])
            if _bad_blocks(a[j:j + 1], xj[None]).numel():
                eye = torch.eye(a.shape[-1], dtype=a.dtype, device=a.device)
                xj = torch.linalg.solve(a[j], eye)
                if _bad_blocks(a[j:j + 1], xj[None]).numel():
                    raise RuntimeError("velocity solve: an interior block could not be inverted accurately")
            x[j] = xj
        out[i:i + max_batch] = x
    return out


class VelocityJacobianSolver:
    """x = J^-1 b for the velocity Jacobian J of one linearisation, J given by its condensation pieces."""

    def __init__(self, P, nex, ney, device, interior="nested", sweep="cr", ncomp=2):
        """ncomp: unknowns per node -- 2 for the velocity pair [u | v], 1 for a scalar operator
        (the convection-diffusion Jacobian, or the pressure stiffness of the Schur preconditioner).
        interior: elimination of the element-column interiors ("nested" static condensation, or
        one dense block per column: "lu" factors, "inverse" explicit inverses).  sweep: solve of the
        block-tridiagonal interface system ("cr": block cyclic reduction, about 2 log2(N_ex) batched
        launches; "thomas": block Thomas, 2 N_ex sequential steps)."""
        if P < 1 or nex < 1 or ney < 1:
            raise ValueError("bad mesh")
        if interior not in ("nested", "lu", "inverse"):
            raise ValueError("interior must be 'nested', 'lu' or 'inverse'")
        if sweep not in ("cr", "thomas"):
            raise ValueError("sweep must be 'cr' or 'thomas'")
        if ncomp not in (1, 2):
            raise ValueError("ncomp must be 1 or 2")
        self.sweep, self.ncomp = sweep, ncomp
        self.P, self.nex, self.ney = P, nex, ney
        self.NY, self.NX = ney * P + 1, nex * P + 1
        self.m = ncomp * self.NY
        self.nI = (P - 1) * self.m
        self.device = torch.device(device)
        self.interior = interior
        self.factored = False
        # SEM_PROFILE_FACTOR=1: per-phase wall times of the factorisation (device-synchronised)
        self.profile = os.environ.get("SEM_PROFILE_FACTOR", "") == "1"
        self.timing = {}

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
        """Assemble and factor.  fill(blocks, cols) writes the pieces (sem_velocity_blocks) with
        blocks["AII"] holding the dense interiors of element columns cols = (c0, c1).  When the whole
        mesh's A_II fits in budget_bytes this is one fill + factor(); otherwise (cfg5: 1.17 TB of
        dense interiors at 128^2, P = 12) the nested condensation runs a chunk of columns at a time,
        each chunk's A_II assembled, condensed and freed before the next."""
        per_col = self.nI * self.nI * 8 + 3 * self.nI * 2 * self.m * 8   # A_II + A_IB, W, work per column
        if self.P == 1 or self.nex * per_col <= budget_bytes:
            blocks = self.empty_blocks()
            fill(blocks, (0, self.nex))
            return self.factor(blocks.pop("AII"), **blocks)
        if self.interior != "nested":
            raise ValueError("column-chunked factorisation needs interior='nested'")
        chunk = max(1, int(budget_bytes // per_col))
        blocks = self.empty_blocks(with_interior=False)
        self._nested_index()
        P, nex, ney, m = self.P, self.nex, self.ney, self.m
        ni, ne1, n_e = self._pi.shape[1], self._ne1, self._pe.numel()
        z = dict(dtype=torch.float64, device=self.device)
        Xi, Yie = torch.empty((nex, ney, ni, ni), **z), torch.empty((nex, ney, ni, 2 * ne1), **z)
        Aei, Sinv = torch.empty((nex, ney, 2 * ne1, ni), **z), torch.empty((nex, n_e, n_e), **z)
        S_diag = S_up = S_lo = None
        for c0 in range(0, nex, chunk):
            c1 = min(nex, c0 + chunk)
            with self._phase("fill"):
                blocks["AII"] = torch.zeros((c1 - c0, self.nI, self.nI), **z)
                fill(blocks, (c0, c1))
                AII = blocks.pop("AII")
            Xi[c0:c1], Yie[c0:c1], Aei[c0:c1], Sinv[c0:c1] = self._nested_pieces(AII)
            del AII
            if S_diag is None:   # every fill writes the line pieces in full: take them from the first
                aIB, aBI = blocks["aIB"], blocks["aBI"]
                S_diag = blocks["D"].clone()
                S_up, S_lo = torch.diag_embed(blocks["E"]), torch.diag_embed(blocks["F"])
            self._Xi, self._Yie, self._Aei, self._Se_inv = Xi, Yie, Aei, Sinv
            with self._phase("W"):
                AIB = torch.diag_embed(aIB[c0:c1]).permute(0, 1, 3, 2, 4).reshape(c1 - c0, self.nI, 2 * m)
                W = self._nested_solve(AIB, slice(c0, c1))
                del AIB
            with self._phase("coupling"):
                C = self._interface_coupling(aBI[c0:c1], W)
                del W
                S_diag[c0:c1] -= C[:, 0, :, 0, :]
                S_diag[c0 + 1:c1 + 1] -= C[:, 1, :, 1, :]
                S_up[c0:c1] -= C[:, 0, :, 1, :]
                S_lo[c0:c1] -= C[:, 1, :, 0, :]
                del C
        self._nested_finish()
        self.W = None
        self.aBI, self.aIB = aBI, aIB
        with self._phase("sweep_factor"):
            self._sweep_factor(S_diag, S_up, S_lo)

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
        if P > 1:
            # dense A_IB (nex, nI, 2m): rows (l, r), column block s holds aIB[e, l, s, r] on its diagonal
            AIB = torch.diag_embed(aIB).permute(0, 1, 3, 2, 4).reshape(nex, self.nI, 2 * m)
            if self.interior == "nested":
                self._nested_factor(AII)
                del AII
                W = self._nested_solve(AIB)
            else:
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
            self.W = W.view(nex, self.nI, 2, m) if self.interior != "nested" else None
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
        # block Thomas on the interface lines: Dt[0] = S_diag[0], Uh[L] = Dt[L]^-1 S_up[L],
        # Dt[L+1] = S_diag[L+1] - S_lo[L] Uh[L]; explicit (pivoted) inverses of the pivot blocks
        Dinv = torch.empty((nex + 1, m, m), dtype=torch.float64, device=self.device)
        Uh = torch.empty((nex, m, m), dtype=torch.float64, device=self.device)
        Dt = S_diag[0]
        for L in range(nex + 1):
            if L > 0:
                Dt = S_diag[L] - S_lo[L - 1] @ Uh[L - 1]
            Dinv[L] = torch.linalg.inv(Dt)
            if L < nex:
                Uh[L] = Dinv[L] @ S_up[L]
        self.Dinv, self.Uh, self.S_lo = Dinv, Uh, S_lo
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

    def _cr_solve_hip(self, g):
        import ctypes as C
        from .. import _lib
        lib = _lib.load()
        m = g.shape[1]
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        x = torch.zeros_like(g)
        P = C.c_void_p

        def gemv(M, srcs, xrow, y, yrow, acc):
            S = len(srcs)
            if not (M.is_contiguous() and xrow.is_contiguous() and yrow.is_contiguous()
                    and xrow.dtype == yrow.dtype == torch.int64 and tuple(M.shape) == (yrow.numel(), m, S * m)
                    and tuple(xrow.shape) == (S, yrow.numel())):
                raise ValueError("sem_block_gemv: operator / index layout")
            if S * m > GEMV_LDS_DOUBLES:   # operands beyond the kernel's LDS staging (cfg5: m = 3074): batched GEMV
                rhs = torch.cat([torch.where((r >= 0)[:, None], t[r.clamp(min=0)], 0.0) for t, r in zip(srcs, xrow)],
                                dim=1)
                out = torch.bmm(M, rhs[..., None])[..., 0]
                if acc:
                    y[yrow] += out
                else:
                    y[yrow] = out
                return
            src = (P * S)(*(P(t.data_ptr()) for t in srcs))
            ld = (C.c_int64 * S)(*(t.stride(0) for t in srcs))
            _lib.check(lib.sem_block_gemv(yrow.numel(), m, S, P(M.data_ptr()), src, ld, P(xrow.data_ptr()),
                                          P(y.data_ptr()), y.stride(0), P(yrow.data_ptr()), int(acc), stream))
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

    def _nested_pieces(self, AII):
        """Element-interior inverses Xi, Xi A_ie, A_ei and the inverse edge Schur blocks of the
        columns whose dense interiors AII holds."""
        nex, ney = AII.shape[0], self.ney
        pi, pe, pel = self._pi, self._pe, self._pe_el
        e = torch.arange(nex, device=self.device)[:, None, None, None]
        with self._phase("gather"):
            A_ii = AII[e, pi[None, :, :, None], pi[None, :, None, :]]     # (nex, ney, ni, ni)
            A_ie = AII[e, pi[None, :, :, None], pel[None, :, None, :]]    # (nex, ney, ni, 2 ne1)
            A_ei = AII[e, pel[None, :, :, None], pi[None, :, None, :]]    # (nex, ney, 2 ne1, ni)
            S_e = AII[e[:, :, 0], pe[None, :, None], pe[None, None, :]]   # (nex, n_e, n_e)
        with self._phase("inv_element"):
            Xi = batched_inverse(A_ii.reshape(-1, *A_ii.shape[-2:])).view(A_ii.shape)
        with self._phase("edge_schur"):
            Yie = Xi @ A_ie
            C = (A_ei @ Yie).view(nex, ney, 2, self._ne1, 2, self._ne1)
            S = S_e.view(nex, ney + 1, self._ne1, ney + 1, self._ne1)
            n = torch.arange(ney, device=self.device)
            for a in range(2):          # element n touches edge rows k = n + a, columns k = n + b
                for b in range(2):
                    S[:, n + a, :, n + b, :] -= C[:, :, a, :, b, :].permute(1, 0, 2, 3)  # index dims lead
        with self._phase("inv_edge"):
            Se_inv = batched_inverse(S_e)
        return Xi, Yie, A_ei, Se_inv

    def _nested_factor(self, AII):
        self._nested_index()
        self._Xi, self._Yie, self._Aei, self._Se_inv = self._nested_pieces(AII)
        self._nested_finish()

    def _nested_finish(self):
        if self.device.type == "cuda":   # column-major blocks for sem_nested_solve (ns_condense.hip)
            self._hipT = tuple(t.transpose(-1, -2).contiguous() for t in
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
        Ye = self._Se_inv[cols] @ Re                                    # (nex, n_e, k)
        Yv = Ye.view(nex, ney + 1, ne1, k)
        Yi = Ti - self._Yie[cols] @ torch.cat((Yv[:, :-1], Yv[:, 1:]), dim=2)
        Y = torch.empty_like(R)
        Y[:, self._pi] = Yi
        Y[:, self._pe] = Ye
        return Y

    # ------------------------------------------------------------------ solve
    def _hip_nested(self):
        """Descriptor and work arrays of sem_nested_solve / sem_interface_rhs (built once)."""
        if getattr(self, "_nd", None) is None:
            from .. import _lib
            nex, ney, P, m = self.nex, self.ney, self.P, self.m
            ni, ne1 = self._pi.shape[1], self._ne1
            z = dict(dtype=torch.float64, device=self.device)
            self._work = (torch.empty(nex * ney * ni, **z), torch.empty(nex * ney * 2 * ne1, **z),
                          torch.empty(nex * (ney + 1) * ne1, **z), torch.empty((nex, self.nI), **z),
                          torch.empty((nex + 1, m), **z))
            T, Cw, Ye, _, _ = self._work
            p = lambda t: t.data_ptr()  # noqa: E731
            XiT, AeiT, YieT, SeT = self._hipT
            self._nd = _lib.SemNestedDesc(P, nex, ney, self.ncomp, self.NY, p(XiT), p(AeiT), p(YieT), p(SeT),
                                          p(self._pi), p(self._pe), p(T), p(Cw), p(Ye))
        return self._nd

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
        _, _, _, yI, g = self._work
        st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        v = C.c_void_p
        b1 = B.data_ptr() + 8 * m   # line e P + 1: first interior line of column e
        _lib.check(lib.sem_nested_solve(C.byref(d), v(b1), P * m, None, None, v(yI.data_ptr()), self.nI, st))
        _lib.check(lib.sem_interface_rhs(P, nex, m, v(B.data_ptr()), m, v(self.aBI.data_ptr()), v(yI.data_ptr()),
                                         self.nI, v(g.data_ptr()), st))
        xB = self._cr_solve(g)
        out = torch.empty((NX, m), dtype=torch.float64, device=self.device)
        out[0::P] = xB
        _lib.check(lib.sem_nested_solve(C.byref(d), v(b1), P * m, v(self.aIB.data_ptr()), v(xB.data_ptr()),
                                        v(out.data_ptr() + 8 * m), P * m, st))
        return out

    def _solve_lines(self, B):
        """x = J^-1 b with b, x as (NX, 2 NY) line arrays (every line: u then v)."""
        P, nex, m, NX = self.P, self.nex, self.m, self.NX
        if (self.device.type == "cuda" and P > 1 and self.interior == "nested" and self.sweep == "cr"
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
        if self.sweep == "cr":
            xB = self._cr_solve(g)
        else:   # block Thomas with the pivot blocks' explicit inverses
            z = torch.empty_like(g)
            z[0] = self.Dinv[0] @ g[0]
            for L in range(1, nex + 1):
                z[L] = self.Dinv[L] @ (g[L] - self.S_lo[L - 1] @ z[L - 1])
            xB = z
            for L in range(nex - 1, -1, -1):
                xB[L] = z[L] - self.Uh[L] @ xB[L + 1]
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
