"""Element-partitioned condensed direct solve (the multi-GPU half of SURVEY.md 8f rank 4, cfg5).

The reference solves its Newton updates in one process (SuperLU, NavierStokes_Solver.py:176-236; its
only parallelism is the two-component ParallelGroup, OpenMDAO/Boussinesq_ParallelCoupler.py:68-100).
Here every rank holds the element columns [eb, ee) of a strip partition (sem_amd/parallel.py) and its
lines eb P .. ee P; neighbouring strips share one interface line.

Factor, per rank (no communication until the last step):
  1. the nested condensation of the rank's own columns (velocity_solve.py, factor_condensed) -- the HIP
     kernel writes the strip's pieces (sem_condensed_blocks on a strip handle: partial rows on the two
     interface lines, the pointwise terms and Dirichlet rows of a shared line left to its right owner),
     giving the strip's block-tridiagonal interface system over its local lines 0..n (n = ee - eb);
  2. the local interface lines 1..n-1 are eliminated by block LU (block Thomas with pivoted pivot-block
     inverses), keeping the two strip-boundary lines: a 2 x 2 block system R (m x m blocks) per rank;
  3. the R of all ranks are all-gathered (RCCL under "nccl") and every rank factors the reduced
     block-tridiagonal system over the G + 1 strip-boundary lines (block cyclic reduction), whose
     shared-line blocks are the sums of the two neighbours' partial blocks.
Solve of J x = b (b on the rank's lines, equal on shared lines): interior solves of the own columns,
the interface right-hand side (a shared line's b counted by its right owner only), local forward
elimination to the two boundary lines, ONE all-gather of 2 m doubles per rank, the replicated reduced
solve, local back substitution, interior back substitution.  x comes out on every rank's lines, equal
on shared lines.

The reduced system over the strip-boundary lines (step 3 and the solve's all-gather + GEMV) and the agreed graph
capture live in `_StripReduced`, which the NS velocity solve's default strip solver shares:
nested_dissection.StripNDSolver eliminates each strip by nested dissection instead of by lines and hands the same
reduced system its Schur complement on the strip's two interface lines.  StripLineSolver stays the strip solver of
the other Dirichlet sets (the CD Jacobian's W / E rows).
"""
import os

import torch

from ..tracing import phase
from .velocity_solve import (VelocityJacobianSolver, _gemv, _gemv2, fused_thomas_operators, fused_thomas_solve,
                             pivot_inverse, twisted_thomas_operators, twisted_thomas_solve, twisted_thomas_solve_mat)


class _StripReduced:
    """The part of an element-partitioned solve that the strips share, whatever eliminates each strip's interior:
    the strip attributes, the all-gather, the reduced block-tridiagonal system over the G + 1 strip-boundary lines
    (this rank's two block rows of its inverse), its solve, and the graph capture agreed by every rank.  Mixed into
    StripLineSolver (line condensation) and nested_dissection.StripNDSolver."""

    def _strip_init(self, nex, bounds, rank, dist, group, gather_device):
        eb, ee = bounds[rank], bounds[rank + 1]
        self.nex_global, self.eb, self.ee = nex, eb, ee
        self.bounds, self.rank, self.G = list(bounds), rank, len(bounds) - 1
        self.dist, self.group = dist, group
        self.gather_device = torch.device(gather_device) if gather_device is not None else self.device
        self.own_right = ee >= nex     # a shared right line belongs to the strip on its right
        # the reduced system over the G + 1 strip-boundary lines: "rows" (default) keeps this rank's two block rows
        # of its inverse (one GEMV per solve); "cr" factors and solves it whole on every rank (round 4, A/B)
        self.reduced = os.environ.get("SEM_STRIP_REDUCED", "rows")

    def _probe_lines(self):
        """This strip's lines eb P .. ee P among the mesh's nex P + 1 (refinement probes agree on shared lines)."""
        return self.eb * self.P, self.ee * self.P + 1, self.nex_global * self.P + 1

    def _all_gather(self, t):
        """[t of rank 0, ..., t of rank G-1] (same shape everywhere) on this solver's device."""
        if self.G == 1:
            return [t]
        src = t.to(self.gather_device).contiguous()
        out = [torch.empty_like(src) for _ in range(self.G)]
        self.dist.all_gather(out, src, group=self.group)
        return [o.to(self.device) for o in out]

    def _reduced_factor(self, R):
        """The reduced system over the G + 1 strip-boundary lines from every strip's 2 x 2 block system R (its
        Schur complement on its two boundary lines), factored on every rank."""
        m = self.m
        dev, f64 = self.device, torch.float64
        Rs = self._all_gather(R)
        G = self.G
        Rd = torch.zeros((G + 1, m, m), dtype=f64, device=dev)
        Ru = torch.empty((G, m, m), dtype=f64, device=dev)
        Rl = torch.empty((G, m, m), dtype=f64, device=dev)
        for j, Rj in enumerate(Rs):
            Rd[j] += Rj[0, 0]
            Rd[j + 1] += Rj[1, 1]
            Ru[j], Rl[j] = Rj[0, 1], Rj[1, 0]
        del Rs
        self._red = self._Z = None
        if self.reduced == "cr":     # round-4 form: every rank factors and solves the whole reduced system
            red = VelocityJacobianSolver(1, G, 1, dev)
            red.m = m
            red._cr_factor(Rd, Ru, Rl)
            self._red = red
        else:
            self._Z = self._reduced_rows(Rd, Ru, Rl)
        self.factored = True

    def _reduced_rows(self, Rd, Ru, Rl):
        """Z = block rows r, r+1 of R^-1 for this rank r (2m x (G+1)m): the solve then needs x_r, x_{r+1} = Z h as ONE
        streaming GEMV instead of a replicated solve of the whole reduced system (round 4: block cyclic reduction on
        every rank, 3.9 ms per cfg5 matvec at G = 8 -- as long as the rest of the strip's solve,
        tools/strip_profile.py).  R is eliminated from line 0 down to r - 1 and from line G up to r + 2, leaving
        the 2 x 2 block system M of lines r, r+1:
          top     Dt_0 = Rd[0],  Dt_j = Rd[j] - Rl[j-1] Dt_{j-1}^-1 Ru[j-1];  line r's right-hand side
                  h_r + sum_{j<r} A_j h_j,  A_{r-1} = -Rl[r-1] Dt_{r-1}^-1,  A_j = A_{j+1} (-Rl[j] Dt_j^-1)
          bottom  Et_G = Rd[G],  Et_j = Rd[j] - Ru[j] Et_{j+1}^-1 Rl[j];  line r+1's
                  h_{r+1} + sum_{j>r+1} B_j h_j,  B_{r+2} = -Ru[r+1] Et_{r+2}^-1,  B_{j+1} = B_j (-Ru[j] Et_{j+1}^-1)
          Z = M^-1 [A_0 .. A_{r-1} I 0 0 .. 0; 0 .. 0 0 I B_{r+2} .. B_G]
        (Ru[j]: row j <- j+1, Rl[j]: row j+1 <- j.)  Factor cost: G pivot inverses and ~2G m^3 GEMMs."""
        G, r, m = self.G, self.rank, self.m
        inv = pivot_inverse
        dev, f64 = self.device, torch.float64
        Z = torch.zeros((2 * m, (G + 1) * m), dtype=f64, device=dev)
        A, Dt_inv = [], None
        for j in range(r):   # top chain: A_j appended as -Rl[j] Dt_j^-1 (products formed below)
            D = Rd[j] if j == 0 else Rd[j] - Rl[j - 1] @ (Dt_inv @ Ru[j - 1])
            Dt_inv = inv(D)
            A.append(-(Rl[j] @ Dt_inv))
        Mtop = Rd[r] if r == 0 else Rd[r] - Rl[r - 1] @ (Dt_inv @ Ru[r - 1])
        B, Et_inv = {}, None
        for j in range(G, r + 1, -1):   # bottom chain
            E = Rd[j] if j == G else Rd[j] - Ru[j] @ (Et_inv @ Rl[j])
            Et_inv = inv(E)
            B[j] = -(Ru[j - 1] @ Et_inv)
        Mbot = Rd[r + 1] if r + 1 == G else Rd[r + 1] - Ru[r + 1] @ (Et_inv @ Rl[r + 1])
        M = torch.cat((torch.cat((Mtop, Ru[r]), dim=1), torch.cat((Rl[r], Mbot), dim=1)), dim=0)
        Mi = inv(M)
        Z[:, r * m:(r + 1) * m] = Mi[:, :m]
        Z[:, (r + 1) * m:(r + 2) * m] = Mi[:, m:]
        P = Mi[:, :m]
        for j in range(r - 1, -1, -1):   # Z_j = Mi[:, :m] A_{r-1} ... A_j
            P = P @ A[j]
            Z[:, j * m:(j + 1) * m] = P
        P = Mi[:, m:]
        for j in range(r + 2, G + 1):    # Z_j = Mi[:, m:] B_{r+2} ... B_j
            P = P @ B[j]
            Z[:, j * m:(j + 1) * m] = P
        return Z

    def _reduced_solve(self, h):
        """x on this strip's two boundary lines (2m) from every strip's boundary right-hand sides h (2, m): ONE
        all-gather and one streaming GEMV (or the replicated CR solve)."""
        m = self.m
        with phase("strip.allgather"):
            H = torch.stack(self._all_gather(h))      # (G, 2, m): the boundary right-hand sides of every strip
        with phase("strip.reduced_solve"):
            rhs = torch.zeros((self.G + 1, m), dtype=torch.float64, device=self.device)
            rhs[:-1] += H[:, 0]
            rhs[1:] += H[:, 1]
            if self._Z is not None:    # x_r, x_{r+1} = Z h: one streaming GEMV over this rank's rows of R^-1
                xb2 = torch.empty(2 * m, dtype=torch.float64, device=self.device)
                _gemv(self._Z, rhs.reshape(-1), xb2)
            else:
                xb2 = self._red._cr_solve(rhs)[self.rank:self.rank + 2].reshape(-1)
        return xb2

    def capture(self):
        """Graph capture of the solve: only when the reduced system's all-gather runs on the device (RCCL,
        capturable); under gloo the all-gather goes through the host, so the solve stays eager.
        Under RCCL the captured graph is checked against the eager solve before it is used."""
        if self.G > 1 and (self.gather_device.type != "cuda" or os.environ.get("SEM_STRIP_GRAPH", "1") == "0"):
            return False
        captured = super().capture()       # a capture executes no collective: a failure desynchronises no rank
        if self.G == 1:
            return captured
        if not self._agree(captured):
            self._graph = None
            return False
        g = torch.Generator(device=self.device).manual_seed(11)
        b = torch.rand(self._bin.shape, dtype=torch.float64, device=self.device, generator=g)
        want = self._solve_lines(b.clone())
        self._bin.copy_(b)
        self._graph.replay()           # every rank replays: its all-gather needs every rank
        err = (self._xout - want).abs().max() / want.abs().max().clamp(min=1e-300)
        if not self._agree(bool(err <= 1e-12)):
            self._graph = None
            return False
        return True

    def _agree(self, ok):
        """True when every rank reports ok (one all-reduce; every rank takes the same decision)."""
        flag = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=self.gather_device)
        self.dist.all_reduce(flag, op=self.dist.ReduceOp.MIN, group=self.group)
        return float(flag.item()) == 1.0


class StripLineSolver(_StripReduced, VelocityJacobianSolver):
    """x = J^-1 b for a Jacobian whose element columns are strip-partitioned across the ranks of `dist`, each strip
    condensed by lines (module docstring)."""

    def __init__(self, P, nex, ney, device, bounds, rank, dist, group=None, ncomp=2, gather_device=None):
        """bounds: the StripPartition bounds (rank r holds element columns [bounds[r], bounds[r+1]));
        gather_device: where the all-gathered blocks travel (the GPU under RCCL, the host under gloo)."""
        super().__init__(P, bounds[rank + 1] - bounds[rank], ney, device, interior="nested", sweep="auto", ncomp=ncomp)
        self._strip_init(nex, bounds, rank, dist, group, gather_device)

    # ------------------------------------------------------------------ factor
    def factor_mesh(self, mesh, budget_bytes=24 << 30, **kw):
        """Assemble the strip's condensed pieces on its strip handle (HIP) and factor."""
        if mesh.ex_begin != self.eb or mesh.ex_end != self.ee:
            raise ValueError("the mesh handle must hold this rank's strip")
        kw = dict(kw, ncomp=self.ncomp)
        eb = self.eb
        if self.P == 1:
            raise ValueError("the strip solve needs P >= 2")
        return self.factor_condensed(
            lambda b, cols: mesh.condensed_blocks(b, cols=(cols[0] + eb, cols[1] + eb), **kw), budget_bytes)

    def _sweep_factor(self, S_diag, S_up, S_lo):
        """Local lines 0..n: eliminate 1..n-1 (block LU), keep the strip's boundary lines 0 and n.  One
        rank: the whole-mesh sweep."""
        if self.G == 1:
            self._T = None
            return super()._sweep_factor(S_diag, S_up, S_lo)
        n, m = self.nex, self.m
        dev, f64 = self.device, torch.float64
        inv = pivot_inverse
        if n == 1:
            R = torch.stack((torch.stack((S_diag[0], S_up[0])), torch.stack((S_lo[0], S_diag[1]))))
            self._T = None
        elif self.sweep_form == "twisted" and n - 1 >= 3:
            # two-ended sweep of the interior lines, as the whole mesh's; X0, X1 from the same factors (one set of
            # pivot inverses: ADVICE r4 -- the one-ended factors were formed only for X0, X1 and doubled them)
            k = n - 1
            op = twisted_thomas_operators(S_diag[1:n], S_up[1:n - 1], S_lo[1:n - 1])
            rhs = torch.zeros((k, m, 2 * m), dtype=f64, device=dev)
            rhs[0, :, :m] = S_lo[0]
            rhs[k - 1, :, m:] = S_up[n - 1]
            X01 = twisted_thomas_solve_mat(op, rhs)
            del rhs
            X0, X1 = X01[..., :m], X01[..., m:]
            R = torch.stack((torch.stack((S_diag[0] - S_up[0] @ X0[0], -(S_up[0] @ X1[0]))),
                             torch.stack((-(S_lo[n - 1] @ X0[k - 1]), S_diag[n] - S_lo[n - 1] @ X1[k - 1]))))
            self._T = (("twisted", op), X01)
        else:
            k = n - 1                           # interior lines 1..n-1 -> rows 0..k-1 of T
            Dinv = torch.empty((k, m, m), dtype=f64, device=dev)
            Uh = torch.empty((max(k - 1, 1), m, m), dtype=f64, device=dev)
            Dinv[0] = inv(S_diag[1])
            for i in range(1, k):
                Uh[i - 1] = Dinv[i - 1] @ S_up[i]                      # T's upper block of row i-1
                Dinv[i] = inv(S_diag[i + 1] - S_lo[i] @ Uh[i - 1])     # T's lower block of row i
            # X0 = T^-1 [S_lo[0]; 0; ...] (coupling of the interior to line 0), X1 = T^-1 [0; ...; S_up[n-1]]
            X0 = torch.empty((k, m, m), dtype=f64, device=dev)
            X1 = torch.zeros((k, m, m), dtype=f64, device=dev)
            X0[0] = Dinv[0] @ S_lo[0]
            for i in range(1, k):
                X0[i] = -(Dinv[i] @ (S_lo[i] @ X0[i - 1]))
            X1[k - 1] = Dinv[k - 1] @ S_up[n - 1]
            for i in range(k - 2, -1, -1):
                X0[i] -= Uh[i] @ X0[i + 1]
                X1[i] = -(Uh[i] @ X1[i + 1])
            R = torch.stack((torch.stack((S_diag[0] - S_up[0] @ X0[0], -(S_up[0] @ X1[0]))),
                             torch.stack((-(S_lo[n - 1] @ X0[k - 1]), S_diag[n] - S_lo[n - 1] @ X1[k - 1]))))
            # the solve's operators: the fused block-Thomas sweep of the interior lines (one GEMV per line and
            # direction, as the whole-mesh sweep) and [X0 | X1] for the back substitution in one batched GEMV
            th = ("single", fused_thomas_operators(Dinv, S_lo[1:n - 1] if n > 2 else None, Uh[:k - 1]))
            X01 = torch.cat((X0, X1), dim=2)
            del Dinv, Uh, X0, X1
            self._T = (th, X01)
        self._S_up0, self._S_lon = S_up[0].clone(), S_lo[n - 1].clone()
        del S_diag, S_up, S_lo
        self._reduced_factor(R)

    # ------------------------------------------------------------------ solve
    def _own_rhs(self, g, B):
        if not self.own_right:          # the right line's right-hand side is its right owner's
            g[-1] -= B[-1]

    def _thomas(self, g):
        """y = T^-1 g for the local interior lines (g: (k, m)): the fused block-Thomas sweep, two-ended when the
        strip has at least three interior lines."""
        form, op = self._T[0]
        return twisted_thomas_solve(op, g) if form == "twisted" else fused_thomas_solve(*op, g)

    def _iface_solve(self, g):
        """No host synchronisation under RCCL (the all-gather stays on the device): stream-capturable."""
        if self.G == 1:
            return super()._iface_solve(g)
        n = self.nex
        with phase("strip.interior_sweep"):
            if self._T is not None:
                y = self._thomas(g[1:n])
                h = torch.stack((g[0], g[n]))   # the boundary lines' right-hand sides: one dual streaming GEMV
                _gemv2((self._S_up0, y[0], h[0]), (self._S_lon, y[-1], h[1]), alpha=-1.0, beta=1.0)
            else:
                y, h = None, torch.stack((g[0], g[1]))
        xb2 = self._reduced_solve(h)
        m = self.m
        out = torch.empty_like(g)
        out[0], out[n] = xb2[:m], xb2[m:]
        with phase("strip.back_substitution"):
            if y is not None:   # y - X0 x0 - X1 x1 = y - [X0 | X1] [x0; x1]: one streaming GEMV over (k m) x 2m
                X01 = self._T[1]
                out[1:n] = y
                _gemv(X01.view(-1, X01.shape[-1]), xb2, out[1:n].reshape(-1), alpha=-1.0, beta=1.0)
        return out
