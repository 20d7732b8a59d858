"""Nested-dissection (multifrontal) direct solve of the Navier-Stokes velocity Jacobian.

The reference factors the Dirichlet-row-replaced velocity Jacobian with SuperLU (`splu`,
NavierStokes_Solver.py:176-192), whose default column order is COLAMD: a fill-reducing order.  The line
condensation of velocity_solve.py eliminates in line order instead -- every element column's interior, then a
block-tridiagonal system over the N_ex + 1 interface lines whose blocks are DENSE (m x m, m = 2 N_y): 28.9 of
the 42.3 GB a cfg5 solve reads are those line blocks (tools/nd_model.py, profiles/r06/velocity/nd_model.json).
This module orders the same Jacobian by nested dissection of the element grid, the structured-mesh analogue of
a fill-reducing order:

* leaves = elements.  Element e's matrix A_e (the element's share of the assembled operator: the x and y rows
  of its own GLL tables with the element's weights, the mass product, the pointwise Jacobian terms on the
  element that owns the node -- sum_e A_e is the assembled Jacobian) is split into its interior unknowns i
  (ncomp (P-1)^2) and its boundary unknowns b (ncomp 4P); Xi = A_ii^-1, the update U_e = A_bb - A_bi Xi A_ib.
* fronts = separators.  The element grid is bisected recursively along its longer side at the middle element
  edge; the separator S of a piece is the skeleton nodes of that edge line strictly inside the piece, and its
  front also holds B, the piece's perimeter nodes that belong to ancestor separators.  The front matrix over
  [S; B] is the extend-add of its two children's updates; S^-1 is formed (batched, pivoted inside the block)
  and the front keeps Fw = [S^-1; A_BS S^-1] ((|S| + |B|) x |S|) and V = S^-1 A_SB (|S| x |B|), and passes
  U = A_BB - A_BS V to its parent.
* Dirichlet rows (the whole perimeter, every component: the velocity mask of NavierStokes_Solver.py:78-94) are
  identity rows: x_D = b_D.  They are taken out before the elimination -- the right-hand side is lifted,
  b_N -= A_ND b_D (the perimeter elements' coupling blocks), and D appears in no front.
* Split leaves (two components, P <= 12): inside an element u and v couple only through the diagonal Newton
  terms, A_ii = [A_uu D1; D2 A_vv], so the leaf keeps A_uu^-1 and S_v^-1 = (A_vv - D2 A_uu^-1 D1)^-1 -- two
  n x n blocks (n = (P-1)^2) instead of the (2n)^2 of Xi -- and sem_leaf_forward solves y_i = A_ii^-1 b_i with
  A_uu^-1 held in registers across its two products.  A per-element probe of the split solve's backward error
  falls back to Xi for the whole mesh when the coupling rivals the stiffness (SPLIT_ETA).
* Solve = lift, leaf forward (y_i and the sparse boundary update A_bi y_i), front forward level by level from
  the deepest, front back substitution x_S = y_S - V x_B from the root down, leaf back substitution
  x_i = y_i - V_e x_b.  Every front step is one streaming GEMV launch over all fronts of a level
  (sem_front_gemv) plus, after a forward step, one deterministic scatter (sem_front_scatter: each target sums
  its <= 4 contributions in a fixed order), so results are bitwise reproducible and the solve is
  graph-capturable.

Bytes per solve (cfg5: 128^2 elements, P = 12): the split leaves' blobs and V_e, the fronts' Fw and V -- 13.5 GB
(17.2 with Xi leaves) against the line condensation's 42.3 (model: tools/nd_model.py).  Strips use it too
(StripNDSolver).  The algebra runs on any torch device: the CPU path (a per-front loop over the same tables) is
what the CPU tests check against SciPy's sparse solve.
"""
import functools
import math
import os

import numpy as np
import torch

from .strip_solve import _StripReduced
from .velocity_solve import VelocityJacobianSolver, batched_inverse, pivot_inverse

ALL_SIDES = 15   # SEM_SIDE_W | E | S | N


class NDTree:
    """Symbolic analysis of the nested dissection for the element columns [xa, xb) (default: all) of an nex x ney
    mesh of order P, ncomp unknowns per node, the mesh's whole perimeter Dirichlet.  Unknowns are addressed by their
    flat index in the solver's local (NX, ncomp N_y) line array (lines xa P .. xb P): (gx - xa P) m + c N_y + gy
    (m = ncomp N_y).  On a strip (xa > 0 or xb < nex) the root's boundary B is the strip's interface lines: they
    are eliminated by the reduced system the strips share (StripNDSolver)."""

    def __init__(self, P, nex, ney, nc, xa=0, xb=None):
        if P < 2:
            raise ValueError("nested dissection needs P >= 2 (element interiors)")
        xb = nex if xb is None else xb
        if not 0 <= xa < xb <= nex:
            raise ValueError("bad element-column range")
        self.P, self.nex, self.ney, self.nc, self.xa, self.xb = P, nex, ney, nc, xa, xb
        self.NY, self.NX, self.NXg = ney * P + 1, (xb - xa) * P + 1, nex * P + 1
        self.m = nc * self.NY
        NY, NXg, m = self.NY, self.NXg, self.m
        # element-local order: interior (i, c, j) for i, j in 1..P-1 (the condensed layout's order), then the
        # boundary (i, c, j) for the nodes with i or j in {0, P}, x-major
        loc = np.full((P + 1, P + 1, nc), -1, dtype=np.int64)
        pi, pj, pc = [], [], []
        for i in range(1, P):
            for c in range(nc):
                for j in range(1, P):
                    loc[i, j, c] = len(pi)
                    pi.append(i), pj.append(j), pc.append(c)
        self.ni = len(pi)
        for i in range(P + 1):
            for c in range(nc):
                for j in range(P + 1):
                    if i in (0, P) or j in (0, P):
                        loc[i, j, c] = len(pi)
                        pi.append(i), pj.append(j), pc.append(c)
        self.ne = len(pi)
        self.nb = self.ne - self.ni
        self.loc = loc
        # A_bi is sparse: a boundary unknown couples to the P - 1 interior unknowns of its own column (y rows of a
        # horizontal-edge node) or line (x rows of a vertical-edge node), none at a corner; bpat[r] lists them
        bpat = np.zeros((self.nb, P - 1), dtype=np.int64)
        for r in range(self.nb):
            i, j, c = pi[self.ni + r], pj[self.ni + r], pc[self.ni + r]
            if 0 < i < P:
                bpat[r] = loc[i, 1:P, c]
            elif 0 < j < P:
                bpat[r] = loc[1:P, j, c]
        self.bpat = bpat
        self.pos_i, self.pos_j, self.pos_c = (np.asarray(a, dtype=np.int64) for a in (pi, pj, pc))
        E = (xb - xa) * ney
        ex, ey = np.divmod(np.arange(E, dtype=np.int64), ney)      # local element e = (ex - xa) ney + ey
        self.ex, self.ey = ex + xa, ey
        gx = (ex[:, None] + xa) * P + self.pos_i[None, :]           # global line
        gy = ey[:, None] * P + self.pos_j[None, :]
        self.eflat = (gx - xa * P) * m + self.pos_c[None, :] * NY + gy     # (E, ne) local flat index
        self.eD = (gx == 0) | (gx == NXg - 1) | (gy == 0) | (gy == NY - 1)
        self.fronts = []
        self.root = self._rec(xa, xb, 0, ney, 0)
        self.depth = max((f["depth"] for f in self.fronts), default=-1)
        self._child_maps()

    # ------------------------------------------------------------------ symbolic
    def _is_d(self, gx, gy):
        return (gx == 0) | (gx == self.NXg - 1) | (gy == 0) | (gy == self.NY - 1)

    def _flats(self, gx, gy):
        """Local flat indices of nodes (global gx, gy) for every component, node-major then component."""
        c = np.arange(self.nc, dtype=np.int64)
        return ((gx[:, None] - self.xa * self.P) * self.m + c[None, :] * self.NY + gy[:, None]).reshape(-1)

    def _rec(self, x0, x1, y0, y1, depth):
        P, ney = self.P, self.ney
        if x1 - x0 == 1 and y1 - y0 == 1:
            return ("e", (x0 - self.xa) * ney + y0)
        if x1 - x0 >= y1 - y0:
            xm = (x0 + x1) // 2
            gy = np.arange(y0 * P + 1, y1 * P, dtype=np.int64)
            gx = np.full_like(gy, xm * P)
            c0, c1 = self._rec(x0, xm, y0, y1, depth + 1), self._rec(xm, x1, y0, y1, depth + 1)
            # component-major along the line: contiguous runs of the line array
            S = ((xm - self.xa) * P * self.m + np.arange(self.nc, dtype=np.int64)[:, None] * self.NY
                 + gy[None, :]).reshape(-1)
        else:
            ym = (y0 + y1) // 2
            gx = np.arange(x0 * P + 1, x1 * P, dtype=np.int64)
            gy = np.full_like(gx, ym * P)
            c0, c1 = self._rec(x0, x1, y0, ym, depth + 1), self._rec(x0, x1, ym, y1, depth + 1)
            S = self._flats(gx, gy)
        # the piece's perimeter nodes on ancestor separators (the domain perimeter is Dirichlet: not a front node)
        nodes = []
        ys = np.arange(y0 * P, y1 * P + 1, dtype=np.int64)
        xs = np.arange(x0 * P, x1 * P + 1, dtype=np.int64)
        if x0 > 0:
            nodes.append(np.stack((np.full_like(ys, x0 * P), ys), 1))
        if x1 < self.nex:
            nodes.append(np.stack((np.full_like(ys, x1 * P), ys), 1))
        if y0 > 0:
            nodes.append(np.stack((xs, np.full_like(xs, y0 * P)), 1))
        if y1 < self.ney:
            nodes.append(np.stack((xs, np.full_like(xs, y1 * P)), 1))
        if nodes:
            nd = np.unique(np.concatenate(nodes), axis=0)
            nd = nd[~self._is_d(nd[:, 0], nd[:, 1])]
            B = np.sort(self._flats(nd[:, 0], nd[:, 1]))
        else:
            B = np.zeros(0, dtype=np.int64)
        fid = len(self.fronts)
        self.fronts.append(dict(depth=depth, S=S, B=B, children=(c0, c1)))
        return ("f", fid)

    def _child_maps(self):
        """For every front, each child's update rows as positions in the front's [S; B] order (-1: Dirichlet)."""
        for f in self.fronts:
            key = np.concatenate((f["S"], f["B"]))
            order = np.argsort(key, kind="stable")
            skey = key[order]
            maps = []
            for kind, cid in f["children"]:
                ck = self.eflat[cid, self.ni:] if kind == "e" else self.fronts[cid]["B"]
                p = np.searchsorted(skey, ck)
                p = np.minimum(p, len(skey) - 1)
                hit = skey[p] == ck
                pos = np.where(hit, order[p], -1)
                if kind == "e":
                    if np.any(~hit & ~self.eD[cid, self.ni:]):
                        raise AssertionError("nested dissection: an element boundary node outside its parent front")
                elif not hit.all():
                    raise AssertionError("nested dissection: a child front's boundary outside its parent front")
                maps.append(pos)
            f["maps"] = maps

    def split_perm(self):
        """The interior positions of the u nodes, then the v nodes (element-local order (i, c, j): a component's
        interior block is every other run of P - 1)."""
        return np.concatenate([self.loc[1:self.P, 1:self.P, c].reshape(-1) for c in range(self.nc)])

    def bytes_per_solve(self, split=False):
        """Operator bytes one solve reads: lift, leaves (Xi -- or, split, the per-component blob A_uu^-1, S_v^-1,
        D1, D2 -- the sparse A_bi, V_e), fronts (Fw, V)."""
        E = (self.xb - self.xa) * self.ney
        nper = int(np.any(self.eD[:, self.ni:], axis=1).sum())
        n = (self.P - 1) ** 2
        ld = n + (n & 1)
        fwd = 2 * n * ld + 2 * ld if split else self.ni * self.ni
        leaf = E * (fwd + self.nb * (self.P - 1) + self.ni * self.nb)
        fr = sum(len(f["S"]) * (len(f["S"]) + 2 * len(f["B"])) for f in self.fronts)
        return 8 * (nper * self.ne * self.nb + leaf + fr)


@functools.lru_cache(maxsize=8)
def nd_tree(P, nex, ney, nc, xa=0, xb=None):
    return NDTree(P, nex, ney, nc, xa, xb)


def element_matrices(tree, elems, dx, dy, Ks, Gs, w, c_mass=0.0, c_stiff=0.0, c_gradx=0.0, c_grady=0.0, cu=None,
                     cv=None, juu=None, juv=None, jvu=None, jvv=None, device="cpu"):
    """Element shares A_e (len(elems), ne, ne) of the Jacobian in the tree's element-local order, Dirichlet rows
    zero (their columns kept: the lift reads them).  The operator is the one sem_velocity_blocks writes
    (sem_amd/csrc/ns_velocity.hip): with f_Kx = cK dy/dx, f_Ky = cK dx/dy, f_M = cM dx dy / 4, f_X = cX dy/2,
    f_Y = cY dx/2 and the element-local GLL weights w,
        x row (i, j) -> (k, j): w_j (f_Kx Ks[i][k] + f_X cu(node) Gs[i][k])
        y row (i, j) -> (i, q): w_i (f_Ky Ks[j][q] + f_Y cv(node) Gs[j][q])
        mass: f_M w_i w_j;  juu / jvv on the diagonal, juv / jvu across the components, on the owner element
    -- the element sums of these are the assembled rows (SEM.py:170-245, NavierStokes_Solver.py:123-136)."""
    t = tree
    P, nc, ne = t.P, t.nc, t.ne
    dev = torch.device(device)
    f64 = dict(dtype=torch.float64, device=dev)
    e = torch.as_tensor(np.asarray(elems, dtype=np.int64), device=dev)
    E = e.numel()
    ex, ey = e // t.ney, e % t.ney           # local element column (the strip's vectors are local)
    fKx, fKy = c_stiff * (dy / dx), c_stiff * (dx / dy)
    fM, fX, fY = c_mass * (dx / 2.0) * (dy / 2.0), c_gradx * (dy / 2.0), c_grady * (dx / 2.0)
    Ks, Gs, w = (torch.as_tensor(np.asarray(a), **f64) for a in (Ks, Gs, w))
    n = P + 1
    ar = torch.arange(n, device=dev)
    loc = torch.as_tensor(t.loc, device=dev)                          # (i, j, c) -> position
    node = (ex[:, None, None] * P + ar[None, :, None]) * t.NY + ey[:, None, None] * P + ar[None, None, :]  # (E, i, j)

    def pointwise(v, default):
        if v is None:
            return torch.full((E, n, n), float(default), **f64)
        return v.to(**f64).reshape(-1)[node]

    cuN, cvN = pointwise(cu, 1.0), pointwise(cv, 1.0)
    A = torch.zeros((E, ne * ne), **f64)
    for c in range(nc):
        # x couplings: rows (i, j, c), columns (k, j, c)
        r = loc[:, :, c][:, :, None].expand(n, n, n)                     # (i, j, k)
        col = loc[:, :, c].t()[None, :, :].expand(n, n, n)               # loc[k, j, c] at (i, j, k)
        vx = w[None, None, :, None] * (fKx * Ks[None, :, None, :] + fX * cuN[:, :, :, None] * Gs[None, :, None, :])
        A.scatter_add_(1, (r * ne + col).reshape(1, -1).expand(E, -1), vx.reshape(E, -1))
        # y couplings: rows (i, j, c), columns (i, q, c)
        r = loc[:, :, c][:, :, None].expand(n, n, n)                     # (i, j, q)
        col = loc[:, :, c][:, None, :].expand(n, n, n)                   # loc[i, q, c]
        vy = w[None, :, None, None] * (fKy * Ks[None, None, :, :] + fY * cvN[:, :, :, None] * Gs[None, None, :, :])
        A.scatter_add_(1, (r * ne + col).reshape(1, -1).expand(E, -1), vy.reshape(E, -1))
    own = (((ar[None, :, None] < P) | (ex[:, None, None] + t.xa == t.nex - 1))
           & ((ar[None, None, :] < P) | (ey[:, None, None] == t.ney - 1))).to(torch.float64)   # (E, i, j)
    diag = fM * w[:, None] * w[None, :]
    for c in range(nc):
        d = loc[:, :, c]
        jd = (juu if c == 0 else jvv)
        dv = diag[None].expand(E, n, n).clone()
        if jd is not None:
            dv = dv + own * pointwise(jd, 0.0)
        A.scatter_add_(1, (d * ne + d).reshape(1, -1).expand(E, -1), dv.reshape(E, -1))
        if nc == 2:
            jc = juv if c == 0 else jvu
            if jc is not None:
                o = loc[:, :, 1 - c]
                A.scatter_add_(1, (d * ne + o).reshape(1, -1).expand(E, -1), (own * pointwise(jc, 0.0)).reshape(E, -1))
    A = A.view(E, ne, ne)
    rowD = torch.as_tensor(t.eD, device=dev)[e]                          # (E, ne)
    A.masked_fill_(rowD[:, :, None], 0.0)
    return A


def _gll_tables(P):
    from .. import GLL
    return GLL.standard_stiffness_matrix(P), GLL.standard_gradient_matrix(P), GLL.standard_nodes(P)[1]


class NestedDissectionSolver(VelocityJacobianSolver):
    """x = J^-1 b for the velocity Jacobian J of one linearisation by nested dissection (module docstring).  Same
    interface as VelocityJacobianSolver (solve, solve1, _solve_lines, set_operator, check_refinement, capture);
    factor with factor_mesh(mesh, **kw) (the device mesh) or factor_coeffs(dx, dy, **kw) (any torch device)."""

    def __init__(self, P, nex, ney, device, ncomp=2, cols=None):
        """cols = (xa, xb): the element columns of a strip of the nex x ney mesh (StripNDSolver); the solver's
        lines are then xa P .. xb P."""
        xa, xb = (0, nex) if cols is None else cols
        super().__init__(P, xb - xa, ney, device, interior="nested", sweep="thomas", ncomp=ncomp)
        self.interior = "nd"
        self.tree = nd_tree(P, nex, ney, ncomp, xa, xb)
        self.chunk_elems = int(os.environ.get("SEM_ND_CHUNK", "2048"))

    # ------------------------------------------------------------------ factorisation
    def factor_mesh(self, mesh, budget_bytes=24 << 30, **kw):
        return self.factor_coeffs(mesh.dx, mesh.dy, **kw)

    def factor_coeffs(self, dx, dy, dir_mask=None, dir_sides=ALL_SIDES, ncomp=None, **kw):
        """Factor the Jacobian with coefficients kw (c_mass, c_stiff, c_gradx, c_grady, cu, cv, juu, juv, jvu, jvv;
        the keywords of sem_velocity_blocks) on a mesh of element widths dx, dy; the Dirichlet rows must be the
        whole perimeter (dir_sides = all four, no explicit mask)."""
        if dir_mask is not None or dir_sides != ALL_SIDES:
            raise ValueError("nested dissection needs the whole perimeter Dirichlet (side bits, no mask)")
        n = (self.P - 1) ** 2
        U_leaf = None
        if self.tree.nc == 2 and n <= 121:      # the split leaf (sem_leaf_forward) unless its probe refuses it
            U_leaf = self._factor_leaves(dx, dy, kw, True)
        if U_leaf is None:                      # Xi (sem_front_gemv)
            U_leaf = self._factor_leaves(dx, dy, kw, False)
        t = self.tree
        kind, rid = t.root
        self._root_update = U_leaf[rid].clone() if kind == "e" else None   # a strip's Schur complement on its lines
        self._factor_fronts(U_leaf)
        del U_leaf
        self._build_steps()
        self.factored = True

    # the split leaf's probe bound: its backward error on a random right-hand side per element (explicit A_ii^-1:
    # <= 9e-16 on the oracle's random Jacobians; split: 4.7e-16 at cfg4's Ra = 1e6 state, up to 2e-13 where the
    # Newton coupling rivals the stiffness, i.e. random velocity fields -- those factor with Xi)
    SPLIT_ETA = 4e-15

    def _factor_leaves(self, dx, dy, kw, split):
        """The element leaves: the lift blocks, V_e, the updates U_e (returned), and the forward operators -- split
        (A_uu^-1, S_v^-1, D1, D2 blobs) or Xi; None when the split leaves' probe exceeds SPLIT_ETA."""
        t, dev = self.tree, self.device
        Ks, Gs, w = _gll_tables(self.P)
        E = self.nex * self.ney
        ni, nb, ne = t.ne - t.nb, t.nb, t.ne
        z = dict(dtype=torch.float64, device=dev)
        n = (self.P - 1) ** 2
        self.split = split
        if split:
            self.split_eta = None
        self._leafB = self._leafF = self._leafAc = self._leafV = self._lift = None
        if self.split:
            ld = n + (n & 1)
            self._leafB = torch.zeros((E, 2 * n * ld + 2 * ld + (self.P - 1) * nb), **z)
            perm = t.split_perm()
            pu, pv = (torch.as_tensor(a, device=dev) for a in (perm[:n], perm[n:]))
        else:
            self._leafF = torch.empty((E, ni, ni), **z)          # Xi
            self._leafAc = torch.empty((E, nb, self.P - 1), **z)  # A_bi on its sparsity pattern (tree.bpat)
        bpat = torch.as_tensor(t.bpat, device=dev)
        self._leafV = torch.empty((E, ni, nb), **z)          # Xi A_ib
        U_leaf = torch.empty((E, nb, nb), **z)
        per = np.nonzero(np.any(t.eD[:, ni:], axis=1))[0]    # elements with Dirichlet boundary nodes
        self._per = per
        self._lift = torch.empty((len(per), ne, nb), **z)
        per_slot = np.full(E, -1, dtype=np.int64)
        per_slot[per] = np.arange(len(per))
        eDb = torch.as_tensor(t.eD[:, ni:], device=dev)
        with self._phase("nd_leaves"):
            for e0 in range(0, E, self.chunk_elems):
                e1 = min(E, e0 + self.chunk_elems)
                A = element_matrices(t, np.arange(e0, e1), dx, dy, Ks, Gs, w, device=dev, **kw)
                dcol = eDb[e0:e1]                                      # (q, nb) Dirichlet boundary columns
                ps = per_slot[e0:e1]
                sel = np.nonzero(ps >= 0)[0]
                if len(sel):
                    s_t = torch.as_tensor(sel, device=dev)
                    self._lift[torch.as_tensor(ps[sel], device=dev)] = A[s_t, :, ni:] * dcol[s_t][:, None, :].to(
                        torch.float64)
                A[:, :, ni:].masked_fill_(dcol[:, None, :], 0.0)        # D columns: lifted, out of the elimination
                Aii, Aib = A[:, :ni, :ni], A[:, :ni, ni:]
                Abi, Abb = A[:, ni:, :ni], A[:, ni:, ni:]
                Ac = torch.gather(Abi, 2, bpat[None].expand(e1 - e0, -1, -1))
                rest = Abi.clone().scatter_(2, bpat[None].expand(e1 - e0, -1, -1), 0.0)
                if bool(rest.abs().max() != 0):
                    raise AssertionError("nested dissection: A_bi has entries outside its line / column pattern")
                if self.split:
                    try:
                        V, eta = self._split_leaves(self._leafB[e0:e1], Aii, Aib, Ac, pu, pv)
                    except RuntimeError:        # A_uu or S_v singular (batched_inverse gives up): refused
                        eta = float("inf")
                    if not math.isfinite(eta) or eta > self.SPLIT_ETA:
                        self.split_eta = eta if math.isfinite(eta) else float("inf")
                        return None
                    self.split_eta = max(eta, self.split_eta or 0.0)
                else:
                    Xi = batched_inverse(Aii.contiguous())
                    V = Xi @ Aib
                    self._leafF[e0:e1] = Xi
                    self._leafAc[e0:e1] = Ac
                    del Xi
                self._leafV[e0:e1] = V
                U_leaf[e0:e1] = Abb - Abi @ V
                del A, V
        return U_leaf

    def _blob_views(self, B):
        """(A_uu^-1, S_v^-1, D1, D2, coef^T) views of split-leaf blobs B (q, L) (include/sem_ops.h sem_leaf_forward)."""
        n = (self.P - 1) ** 2
        ld, nb, q = n + (n & 1), self.tree.nb, B.shape[0]
        o = 2 * n * ld
        return (B[:, :n * ld].view(q, n, ld)[:, :, :n], B[:, n * ld:o].view(q, n, ld)[:, :, :n], B[:, o:o + n],
                B[:, o + ld:o + ld + n], B[:, o + 2 * ld:].view(q, self.P - 1, nb))

    def _split_leaves(self, B, Aii, Aib, Ac, pu, pv):
        """Split leaves of one chunk: A_ii = [A_uu D1; D2 A_vv] in [u; v] order (the components couple only through
        the diagonal Newton terms juv, jvu), A_uu^-1 and S_v^-1 = (A_vv - D2 A_uu^-1 D1)^-1 into the blobs B,
        and V_e = A_ii^-1 A_ib by the same block elimination (returned, element-local row order)."""
        Auu, Auv = Aii[:, pu][:, :, pu], Aii[:, pu][:, :, pv]
        Avu, Avv = Aii[:, pv][:, :, pu], Aii[:, pv][:, :, pv]
        d1, d2 = torch.diagonal(Auv, dim1=1, dim2=2), torch.diagonal(Avu, dim1=1, dim2=2)
        if bool((Auv - torch.diag_embed(d1)).abs().max() != 0) or bool((Avu - torch.diag_embed(d2)).abs().max() != 0):
            raise AssertionError("nested dissection: the components couple off the diagonal inside an element")
        Au = batched_inverse(Auu.contiguous())
        Sv = batched_inverse((Avv - d2[:, :, None] * Au * d1[:, None, :]).contiguous())
        Aub, Avb = Aib[:, pu], Aib[:, pv]
        Xv = Sv @ (Avb - d2[:, :, None] * (Au @ Aub))
        V = torch.empty_like(Aib)
        V[:, pv] = Xv
        V[:, pu] = Au @ (Aub - d1[:, :, None] * Xv)
        bAu, bSv, bd1, bd2, bc = self._blob_views(B)
        bAu.copy_(Au)
        bSv.copy_(Sv)
        bd1.copy_(d1)
        bd2.copy_(d2)
        bc.copy_(Ac.transpose(1, 2))
        # probe: the split forward solve of a fixed random right-hand side, backward error per element
        g = torch.Generator(device=Aii.device).manual_seed(7)
        b = torch.rand(Aii.shape[:2], dtype=Aii.dtype, device=Aii.device, generator=g) * 2 - 1
        tt = (Au @ b[:, pu, None])[..., 0]
        yv = (Sv @ (b[:, pv] - d2 * tt)[..., None])[..., 0]
        y = torch.empty_like(b)
        y[:, pv] = yv
        y[:, pu] = tt - (Au @ (d1 * yv)[..., None])[..., 0]
        r = (Aii @ y[..., None])[..., 0] - b
        eta = r.abs().amax(1) / (Aii.abs().sum(2).amax(1) * y.abs().amax(1) + b.abs().amax(1))
        return V, float(eta.max())

    def bytes_per_solve(self):
        return self.tree.bytes_per_solve(self.split)

    def _factor_fronts(self, U_leaf):
        """Fronts by depth (deepest first), batched per (|S|, |B|) shape group."""
        t, dev = self.tree, self.device
        z = dict(dtype=torch.float64, device=dev)
        self._fw = [None] * len(t.fronts)      # (group tensor, slot) of Fw
        self._fv = [None] * len(t.fronts)      # (group tensor, slot) of V
        fu = [None] * len(t.fronts)            # (group tensor, slot) of U
        by_depth = {}
        for fid, f in enumerate(t.fronts):
            by_depth.setdefault(f["depth"], {}).setdefault((len(f["S"]), len(f["B"])), []).append(fid)
        with self._phase("nd_fronts"):
            for depth in sorted(by_depth, reverse=True):
                for (s, b), fids in sorted(by_depth[depth].items()):
                    nf, n = len(fids), s + b
                    F = torch.zeros(nf * n * n + 1, **z)           # + 1: the Dirichlet sink
                    with self._phase(f"nd_extend_add_d{depth}"):
                        for k in range(2):
                            self._extend_add(F, n, fids, k, U_leaf, fu)
                    F = F[:-1].view(nf, n, n)
                    Ass = F[:, :s, :s]
                    with self._phase(f"nd_inverse_d{depth}"):
                        if s >= 1024:
                            Sinv = torch.stack([pivot_inverse(Ass[q].contiguous()) for q in range(nf)])
                        else:
                            Sinv = batched_inverse(Ass.contiguous())
                    Fw = torch.empty((nf, n, s), **z)
                    Fw[:, :s] = Sinv
                    if b:
                        Abs, Asb, Abb = F[:, s:, :s], F[:, :s, s:], F[:, s:, s:]
                        Fw[:, s:] = Abs @ Sinv
                        V = Sinv @ Asb
                        U = Abb - Abs @ V
                    else:
                        V = U = None
                    del F, Sinv
                    for q, fid in enumerate(fids):
                        self._fw[fid] = (Fw, q)
                        self._fv[fid] = (V, q) if b else None
                        fu[fid] = (U, q) if b else None
                        if t.root == ("f", fid) and b:
                            self._root_update = U[q]
                # children's updates are no longer needed once every front of this depth has its matrix
                for fid in [f for g in by_depth[depth].values() for f in g]:
                    for kind, cid in t.fronts[fid]["children"]:
                        if kind == "f":
                            fu[cid] = None

    def _extend_add(self, F, n, fids, k, U_leaf, fu):
        """F[slot] += child k's update of every front of the group, scattered by the child's position map (distinct
        destinations within one call; the Dirichlet rows / columns go to the sink entry F[-1], never read)."""
        t, dev = self.tree, self.device
        sink = F.numel() - 1
        groups = {}
        for q, fid in enumerate(fids):
            kind, cid = t.fronts[fid]["children"][k]
            src = ("leaf", None) if kind == "e" else (id(fu[cid][0]), fu[cid][0])
            groups.setdefault(src[0], (src[1], []))[1].append((q, kind, cid))
        for _, (Ut, items) in groups.items():
            for c0 in range(0, len(items), 4096):
                part = items[c0:c0 + 4096]
                q = torch.as_tensor([it[0] for it in part], device=dev)
                if part[0][1] == "e":
                    cids = [it[2] for it in part]
                    src = U_leaf[torch.as_tensor(cids, device=dev)]
                else:
                    src = Ut[torch.as_tensor([fu[it[2]][1] for it in part], device=dev)]
                pos = torch.as_tensor(np.stack([t.fronts[fids[it[0]]]["maps"][k] for it in part]), device=dev)
                bad = pos < 0
                dest = q[:, None, None] * (n * n) + pos[:, :, None] * n + pos[:, None, :]
                dest = dest.masked_fill(bad[:, :, None] | bad[:, None, :], sink)
                # index_add_ (atomic adds, no sort): every destination but the sink receives one value per call, so the
                # sums are deterministic.  index_put_(accumulate=True) sorted the indices and, with four processes
                # sharing one GPU, spent up to a minute per level in its temporaries (profiles/r06/strip/)
                F.index_add_(0, dest.reshape(-1), src.reshape(-1))

    # ------------------------------------------------------------------ solve plan
    def _build_steps(self):
        """The solve as a list of steps over flat line-array indices: ("fwd", launch, scatter, sparse) and
        ("back", launch).  A launch is a list of (operator tensor T, slot q, xidx, out) per front, the operator T[q]
        (R x K): fwd writes stage[out:out+R], back subtracts from W[out indices]; `sparse` (leaves only) then forms
        the boundary rows from the stage (sem_front_sparse_rows) before the scatter."""
        t = self.tree
        ni, ne = t.ni, t.ne
        steps = []
        # lift: W_N -= A_ND b_D over the perimeter elements
        if len(self._per):
            items, tgt, src = [], [], []
            for q, e in enumerate(self._per):
                items.append((self._lift, q, t.eflat[e, ni:], q * ne))
                keep = ~t.eD[e]
                tgt.append(t.eflat[e][keep])
                src.append(q * ne + np.nonzero(keep)[0])
            steps.append(("fwd", items, self._scatter_plan(np.zeros(0, np.int64), np.zeros(0, np.int64),
                                                           np.concatenate(tgt), np.concatenate(src)), None))
        # leaves forward: y_i = A_ii^-1 b_i and the sparse A_bi y_i into stage[e ne + (ni .. ne)]; split: one
        # sem_leaf_forward (y_i straight to W), else Xi b_i into stage[e ne + (0 .. ni)] and sem_front_sparse_rows
        E = self.nex * self.ney
        items, ct, cs, bt, bs = [], [], [], [], []
        for e in range(E):
            if not self.split:
                items.append((self._leafF, e, t.eflat[e, :ni], e * ne))
                ct.append(t.eflat[e, :ni])
                cs.append(e * ne + np.arange(ni))
            keep = ~t.eD[e, ni:]
            bt.append(t.eflat[e, ni:][keep])
            bs.append(e * ne + ni + np.nonzero(keep)[0])
        none = np.zeros(0, np.int64)
        if self.split:
            n = (self.P - 1) ** 2
            perm = t.split_perm()
            inv = np.empty_like(perm)
            inv[perm] = np.arange(len(perm))
            steps.append(("leaf", dict(iidx=t.eflat[:, perm], pat=inv[t.bpat.T], n=n, nb=t.nb, nelem=E, sstride=ne,
                                       soff=ni),
                          self._scatter_plan(none, none, np.concatenate(bt), np.concatenate(bs)), None))
        else:
            steps.append(("fwd", items, self._scatter_plan(np.concatenate(ct), np.concatenate(cs),
                                                           np.concatenate(bt), np.concatenate(bs)),
                          dict(coef=self._leafAc, pat=t.bpat, stride=ne, out_off=ni, nitems=E)))
        levels = {}
        for fid, f in enumerate(t.fronts):
            levels.setdefault(f["depth"], []).append(fid)
        for depth in sorted(levels, reverse=True):
            items, ct, cs, bt, bs = [], [], [], [], []
            off = 0
            for fid in levels[depth]:
                f = t.fronts[fid]
                s, b = len(f["S"]), len(f["B"])
                Fw, q = self._fw[fid]
                items.append((Fw, q, f["S"], off))
                ct.append(f["S"])
                cs.append(off + np.arange(s))
                bt.append(f["B"])
                bs.append(off + s + np.arange(b))
                off += s + b
            steps.append(("fwd", items, self._scatter_plan(np.concatenate(ct), np.concatenate(cs),
                                                           np.concatenate(bt), np.concatenate(bs)), None))
        for depth in sorted(levels):
            items = []
            for fid in levels[depth]:
                f = t.fronts[fid]
                if len(f["B"]) == 0:
                    continue
                V, q = self._fv[fid]
                items.append((V, q, f["B"], f["S"]))
            if items:
                steps.append(("back", items))
        items = []
        for e in range(E):
            xb = np.where(t.eD[e, ni:], -1, t.eflat[e, ni:])
            items.append((self._leafV, e, xb, t.eflat[e, :ni]))
        steps.append(("back", items))
        self._steps = steps
        self._nfwd = sum(1 for st in steps if st[0] != "back")
        self._stage_len = max(max(max(it[3] + it[0].shape[1] for it in st[1]),
                                  st[3]["nitems"] * st[3]["stride"] if st[3] else 0) if st[0] == "fwd" else
                              st[1]["nelem"] * st[1]["sstride"] for st in steps if st[0] != "back")
        self._hip = self._hip_plan() if self.device.type == "cuda" else None

    @staticmethod
    def _scatter_plan(copy_tgt, copy_src, acc_tgt, acc_src):
        """Copy targets (W[t] = stage[s], one source each) and accumulation targets (W[t] -= sum of stage[s], up to
        four sources, summed in increasing source order)."""
        order = np.lexsort((acc_src, acc_tgt))
        at, asrc = acc_tgt[order], acc_src[order]
        uniq, start, cnt = np.unique(at, return_index=True, return_counts=True)
        if len(cnt) and cnt.max() > 4:
            raise AssertionError("nested dissection: a node with more than four contributions in one step")
        src4 = np.full((len(uniq), 4), -1, dtype=np.int64)
        rank = np.arange(len(at)) - np.repeat(start, cnt)
        src4[np.repeat(np.arange(len(uniq)), cnt), rank] = asrc
        return dict(copy_tgt=copy_tgt.astype(np.int64), copy_src=copy_src.astype(np.int64), acc_tgt=uniq,
                    acc_src=src4)

    # ------------------------------------------------------------------ solve
    def _solve_lines_once(self, B):
        """Forward steps, the strip hook (the reduced system over the strip-boundary lines; nothing on a whole mesh),
        back-substitution steps -- on the device the HIP launches, elsewhere the torch loop over the same tables.
        The working array carries one trailing zero (operand index -1)."""
        Wz = torch.cat((B.reshape(-1), B.new_zeros(1)))
        nf = self._nfwd
        self._run(Wz, 0, nf)
        self._between(Wz[:-1].view(self.NX, self.m), B)
        self._run(Wz, nf, len(self._steps))
        return Wz[:-1].view(self.NX, self.m)

    def _between(self, W, B):
        """After the forward steps: W holds y on every eliminated unknown and the reduced right-hand side on the
        root's boundary (none on a whole mesh)."""

    def _run(self, Wz, lo, hi):
        if self.device.type == "cuda":
            return self._run_hip(Wz, lo, hi)
        stage = Wz.new_zeros(self._stage_len)
        dev = Wz.device
        for st in self._steps[lo:hi]:
            if st[0] == "leaf":     # the split leaves (sem_leaf_forward), batched over the elements
                L = st[1]
                n = L["n"]
                Au, Sv, d1, d2, cT = self._blob_views(self._leafB)
                ii = torch.as_tensor(L["iidx"], device=dev)
                tt = (Au @ Wz[ii[:, :n]][..., None])[..., 0]
                yv = (Sv @ (Wz[ii[:, n:]] - d2 * tt)[..., None])[..., 0]
                y = torch.cat((tt - (Au @ (d1 * yv)[..., None])[..., 0], yv), 1)
                Wz[ii.reshape(-1)] = y.reshape(-1)
                g = (cT * y[:, torch.as_tensor(L["pat"], device=dev)]).sum(1)
                stage[:L["nelem"] * L["sstride"]].view(L["nelem"], -1)[:, L["soff"]:L["soff"] + L["nb"]] = g
            if st[0] in ("fwd", "leaf"):
                for T, q, xidx, off in (st[1] if st[0] == "fwd" else ()):
                    x = Wz[torch.as_tensor(xidx, device=dev)]
                    stage[off:off + T.shape[1]] = T[q] @ x
                sp = st[3]
                if sp is not None:
                    y = stage[:sp["nitems"] * sp["stride"]].view(sp["nitems"], sp["stride"])
                    yi = y[:, torch.as_tensor(sp["pat"], device=dev)]                 # (items, nrows, nnz)
                    y[:, sp["out_off"]:sp["out_off"] + sp["pat"].shape[0]] = (sp["coef"] * yi).sum(-1)
                sc = st[2]
                ct, cs, at, a4 = (torch.as_tensor(sc[k], device=dev) for k in ("copy_tgt", "copy_src", "acc_tgt",
                                                                                "acc_src"))
                Wz[ct] = stage[cs]
                v = Wz[at]
                for k in range(4):
                    s = a4[:, k]
                    v = v - torch.where(s >= 0, stage[s.clamp(min=0)], torch.zeros_like(v))
                Wz[at] = v
            else:
                for T, q, xidx, yidx in st[1]:
                    x = Wz[torch.as_tensor(xidx, device=dev)]
                    y = torch.as_tensor(yidx, device=dev)
                    Wz[y] = Wz[y] - T[q] @ x

    def _hip_plan(self):
        """Device tables of every step (sem_front_gemv descriptors, sem_front_scatter index arrays), checked on the
        host against the line array and the stage buffer before anything is launched."""
        from .. import _lib
        dev = self.device
        nW = self.NX * self.m
        self._stage = torch.zeros(self._stage_len, dtype=torch.float64, device=dev)
        plan = []

        def i32(a):
            a = np.ascontiguousarray(a, dtype=np.int64)
            if a.size and (a.min() < -1 or a.max() >= 2 ** 31 - 1):
                raise AssertionError("nested dissection: index outside int32")
            return torch.as_tensor(a.astype(np.int32), device=dev)

        transposed = {}     # id(group tensor) -> its operators transposed (form 1)
        for st in self._steps:
            if st[0] == "leaf":
                plan.append(self._leaf_plan(st, nW, i32))
                continue
            items, back = st[1], st[0] == "back"
            nf = len(items)
            Ks = np.array([it[0].shape[2] for it in items])
            leaves = any(items[0][0] is t for t in (self._lift, self._leafF, self._leafV))
            form = self._launch_form(back, nf, Ks, leaves)
            ptr = np.empty(nf, dtype=np.int64)
            dims = np.zeros((nf, 4), dtype=np.int64)
            xoff = np.zeros(nf, dtype=np.int64)
            yoff = np.zeros(nf, dtype=np.int64)
            xs, ys = [], []
            xo = yo = 0
            for k, (T, q, xidx, out) in enumerate(items):
                R, K = T.shape[1], T.shape[2]
                if T.stride(2) != 1 or T.stride(1) != K or K % 2 or T.dtype != torch.float64 or T.device != dev:
                    raise AssertionError("nested dissection: operators must be contiguous float64 rows of even length")
                if not 0 <= q < T.shape[0]:
                    raise AssertionError("nested dissection: operator slot outside its group")
                if form == 1:   # A^T, one thread per row
                    Tt = transposed.get(id(T))
                    if Tt is None:
                        Tt = transposed[id(T)] = (T, T.transpose(1, 2).contiguous())
                    ptr[k] = Tt[1].data_ptr() + q * Tt[1].stride(0) * 8
                    dims[k, :3] = (R, K, R)
                else:
                    ptr[k] = T.data_ptr() + q * T.stride(0) * 8
                    if ptr[k] % 16:
                        raise AssertionError("nested dissection: operator rows must be 16-byte aligned")
                    dims[k, :3] = (R, K, K)
                if len(xidx) != K:
                    raise AssertionError("nested dissection: operand count differs from the operator width")
                xoff[k] = xo
                xs.append(xidx)
                xo += K
                if back:
                    if len(out) != R:
                        raise AssertionError("nested dissection: target count differs from the operator height")
                    yoff[k] = yo
                    ys.append(out)
                    yo += R
                else:
                    if out < 0 or out + R > self._stage_len:
                        raise AssertionError("nested dissection: stage overflow")
                    yoff[k] = out
            if int(dims[:, 1].max()) > 8192:
                raise ValueError("nested dissection: a front with more than 8192 operands (sem_front_gemv stages them "
                                 "in LDS); the mesh is too large for this dissection")
            xidx = np.concatenate(xs)
            if xidx.size and (xidx.min() < -1 or xidx.max() >= nW):
                raise AssertionError("nested dissection: operand index outside the line array")
            if back:
                yidx = np.concatenate(ys)
                if yidx.min() < 0 or yidx.max() >= nW or len(np.unique(yidx)) != len(yidx):
                    raise AssertionError("nested dissection: back-substitution targets must be distinct line entries")
            R = dims[:, 0]
            if form == 1:
                lanes, rows = 1, 256
            elif form == 2:
                lanes, rows = 64, 8
            else:
                lanes, rows = self._launch_shape(dims[:, 1], R)
            nt = (R + rows - 1) // rows
            tiles = np.stack((np.repeat(np.arange(nf), nt),
                              np.concatenate([np.arange(n) * rows for n in nt])), 1)
            keep = dict(ptr=torch.as_tensor(ptr, device=dev), dims=i32(dims), xoff=torch.as_tensor(xoff, device=dev),
                        yoff=torch.as_tensor(yoff, device=dev), tiles=i32(tiles), xidx=i32(xidx),
                        yidx=i32(yidx) if back else None, transposed=[v[1] for v in transposed.values()])
            transposed = {}
            d = _lib.SemFrontLaunch(len(tiles), rows, lanes, int(dims[:, 1].max()), int(back), form,
                                    keep["ptr"].data_ptr(),
                                    keep["dims"].data_ptr(), keep["xoff"].data_ptr(), keep["yoff"].data_ptr(),
                                    keep["tiles"].data_ptr(), keep["xidx"].data_ptr(),
                                    keep["yidx"].data_ptr() if back else None, None,
                                    None if back else self._stage.data_ptr())
            sc = None if back else self._scatter_tables(st[2], nW, i32)
            sp = None
            if not back and st[3] is not None:
                q = st[3]
                coef, pat = q["coef"], np.asarray(q["pat"])
                nrows, nnz = pat.shape
                if (tuple(coef.shape) != (q["nitems"], nrows, nnz) or not coef.is_contiguous() or pat.min() < 0
                        or pat.max() >= q["out_off"] or q["out_off"] + nrows > q["stride"]
                        or q["nitems"] * q["stride"] > self._stage_len):
                    raise AssertionError("nested dissection: bad sparse boundary step")
                # the kernel reads coefficient q of every row together: (items, nnz, nrows) and (nnz, nrows)
                sp = dict(nitems=q["nitems"], nrows=nrows, nnz=nnz, coef=coef.transpose(1, 2).contiguous(),
                          pat=i32(pat.T), stride=q["stride"], out_off=q["out_off"])
            plan.append((d, keep, sc, sp))
        return plan

    def _scatter_tables(self, p, nW, i32):
        for a, hi in ((p["copy_tgt"], nW), (p["acc_tgt"], nW)):
            if a.size and (a.min() < 0 or a.max() >= hi):
                raise AssertionError("nested dissection: scatter target outside the line array")
        for a in (p["copy_src"], p["acc_src"]):
            if a.size and (a.min() < -1 or a.max() >= self._stage_len):
                raise AssertionError("nested dissection: scatter source outside the stage")
        if len(np.unique(np.concatenate((p["copy_tgt"], p["acc_tgt"])))) != len(p["copy_tgt"]) + len(p["acc_tgt"]):
            raise AssertionError("nested dissection: scatter targets must be distinct")
        return dict(n_copy=len(p["copy_tgt"]), ct=i32(p["copy_tgt"]), cs=i32(p["copy_src"]), n_acc=len(p["acc_tgt"]),
                    at=i32(p["acc_tgt"]), a4=i32(p["acc_src"]).contiguous())

    def _leaf_plan(self, st, nW, i32):
        """The split leaves' sem_leaf_forward descriptor, its tables checked on the host: interior targets distinct
        line entries, boundary patterns inside [y_u; y_v], the boundary rows inside the stage."""
        from .. import _lib
        L, B = st[1], self._leafB
        n, nb, E = L["n"], L["nb"], L["nelem"]
        ld = n + (n & 1)
        iidx, pat = np.asarray(L["iidx"]), np.asarray(L["pat"])
        if (iidx.shape != (E, 2 * n) or iidx.min() < 0 or iidx.max() >= nW or len(np.unique(iidx)) != iidx.size
                or pat.shape != (self.P - 1, nb) or pat.min() < 0 or pat.max() >= 2 * n
                or E * L["sstride"] > self._stage_len or L["soff"] + nb > L["sstride"] or not 1 <= n <= 121
                or B.shape != (E, 2 * n * ld + 2 * ld + (self.P - 1) * nb) or not B.is_contiguous()
                or B.data_ptr() % 16 or B.shape[1] % 2 or B.device != self.device):
            raise AssertionError("nested dissection: bad split-leaf step")
        keep = dict(iidx=i32(iidx), pat=i32(pat))
        d = _lib.SemLeafLaunch(E, n, ld, nb, self.P - 1, B.shape[1], B.data_ptr(), keep["iidx"].data_ptr(),
                               keep["pat"].data_ptr(), None, self._stage.data_ptr(), L["sstride"], L["soff"])
        return d, keep, self._scatter_tables(st[2], nW, i32), None

    def _launch(self, lib, entry, Wz, st):
        """One planned step on stream st: its gemv (or split-leaf) launch, sparse rows, scatter."""
        import ctypes as C
        from .. import _lib
        d, _, sc, sp = entry
        d.W = Wz.data_ptr()
        if isinstance(d, _lib.SemLeafLaunch):
            _lib.check(lib.sem_leaf_forward(C.byref(d), st))
        else:
            _lib.check(lib.sem_front_gemv(C.byref(d), st))
        if sp is not None:
            _lib.check(lib.sem_front_sparse_rows(sp["nitems"], sp["nrows"], sp["nnz"], sp["coef"].data_ptr(),
                                                 sp["pat"].data_ptr(), self._stage.data_ptr(), sp["stride"],
                                                 sp["out_off"], st))
        if sc is not None:
            _lib.check(lib.sem_front_scatter(sc["n_copy"], sc["ct"].data_ptr(), sc["cs"].data_ptr(), sc["n_acc"],
                                             sc["at"].data_ptr(), sc["a4"].data_ptr(), self._stage.data_ptr(),
                                             Wz.data_ptr(), st))

    def _launch_form(self, back, nf, K, leaves):
        """sem_front_gemv's form for one launch (`forms` = "auto", or "rows" for every launch in form 0): 1 (columns:
        transposed operators, a thread per row) for the forward front levels whose rows are <= 128 doubles (the
        deepest separators: cfg5 d13-d11 124 / 111 / 85 -> 74 / 79 / 71 us, profiles/r06/velocity/nd/; d10-d9
        83 / 63 -> 73 / 56 us, profiles/r06/velocity/split/cols_ab128.json), else 0 (lanes per row).  A k-split form
        for the few long top fronts (operands in registers, four waves per row set) measured slower than form 0
        there (+10-25 %) and was not kept."""
        if getattr(self, "forms", "auto") != "auto" or leaves:
            return 0
        return 1 if not back and int(np.median(K)) <= 128 else 0

    # (lanes per row, rows per workgroup) of sem_front_gemv: (wide, narrow) per lane count
    SHAPES = {64: (16, 4), 32: (16, 8), 16: (32, 16), 8: (64, 32), 4: (128, 64)}

    @classmethod
    def _launch_shape(cls, K, R):
        """Lanes per row from the launch's median row length (pairs per lane ~2-4 on short rows: 64 lanes for rows of
        >= 192 doubles), then the wide tile unless the launch would have fewer than 256 workgroups (the root levels:
        1-2 fronts).  From 256 rather than 2048 on: cfg5 3.054-3.067 -> 3.000-3.003 ms, the top levels' launches of
        384-1918 wide tiles 10-20 % faster; cfg4 unchanged (tools/nd_shapes_ab.py, profiles/r06/velocity/split/)."""
        kp = int(np.median(K)) // 2
        lanes = 64 if kp >= 96 else max(4, min(32, 1 << max(0, (kp // 2).bit_length() - 1)))
        wide, narrow = cls.SHAPES[lanes]
        rows = wide if int(((R + wide - 1) // wide).sum()) >= 256 else narrow
        return lanes, rows

    def _run_hip(self, Wz, lo, hi):
        """Steps lo..hi on the device: one sem_front_gemv per level and direction, the leaves' sparse boundary rows
        (sem_front_sparse_rows), one sem_front_scatter after each forward level (module docstring)."""
        import ctypes as C
        from .. import _lib
        lib = _lib.load()
        st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        for entry in self._hip[lo:hi]:
            self._launch(lib, entry, Wz, st)


class StripNDSolver(_StripReduced, NestedDissectionSolver):
    """The element-partitioned velocity solve with each strip ordered by nested dissection: rank r dissects its own
    element columns [e_b, e_e) with its two interface lines as the root's boundary, so its factor ends in the
    strip's Schur complement on those lines -- its 2 x 2 block system R of the reduced system over the G + 1
    strip-boundary lines that the strips share (strip_solve._StripReduced: one all-gather of R at factor time, this
    rank's two block rows of R^-1, one all-gather of 2m right-hand-side values per solve).  Element shares make the
    partial rows of a shared line automatic (each strip adds its own elements); the Dirichlet identity rows of a
    shared line go to its right owner, and the whole outer lines x = 0, 1 are identity rows.
    Solve: the strip's forward steps (lift, leaves, every level up to its root), the reduced solve for the two
    interface lines, the back-substitution steps -- no coupling solutions X0 / X1 are needed (the fronts' V panels
    carry the interface lines like any ancestor separator)."""

    def __init__(self, P, nex, ney, device, bounds, rank, dist, group=None, ncomp=2, gather_device=None):
        NestedDissectionSolver.__init__(self, P, nex, ney, device, ncomp=ncomp, cols=(bounds[rank], bounds[rank + 1]))
        self._strip_init(nex, bounds, rank, dist, group, gather_device)

    def factor_mesh(self, mesh, budget_bytes=24 << 30, **kw):
        if mesh.ex_begin != self.eb or mesh.ex_end != self.ee:
            raise ValueError("the mesh handle must hold this rank's strip")
        return self.factor_coeffs(mesh.dx, mesh.dy, **kw)

    def factor_coeffs(self, dx, dy, **kw):
        NestedDissectionSolver.factor_coeffs(self, dx, dy, **kw)
        if self.G == 1:
            return
        self._reduced_factor(self._interface_blocks())
        self._root_update = None

    def _interface_blocks(self):
        """R (2, 2, m, m): the root's update U on its boundary (the strip's non-Dirichlet interface-line unknowns)
        placed on the left / right line blocks, plus the identity rows of the lines' Dirichlet unknowns this strip
        owns (its left line; its right line only at the mesh's right end)."""
        t, m, NX, NY = self.tree, self.m, self.NX, self.NY
        kind, rid = t.root
        keys = (t.eflat[rid, t.ni:][~t.eD[rid, t.ni:]] if kind == "e" else t.fronts[rid]["B"])
        U = self._root_update
        if kind == "e":
            U = U[torch.as_tensor(np.nonzero(~t.eD[rid, t.ni:])[0], device=self.device)][
                :, torch.as_tensor(np.nonzero(~t.eD[rid, t.ni:])[0], device=self.device)]
        gxl, r = np.divmod(keys, m)
        if not np.all((gxl == 0) | (gxl == NX - 1)):
            raise AssertionError("nested dissection: a strip root's boundary off its interface lines")
        pos = torch.as_tensor(np.where(gxl == 0, 0, m) + r, device=self.device)
        R = torch.zeros((2 * m, 2 * m), dtype=torch.float64, device=self.device)
        R[pos[:, None], pos[None, :]] = U
        # Dirichlet rows on the lines (both components): all of an outer line, the ends gy = 0, N_y - 1 otherwise
        c_gy = np.arange(m) % NY
        for side, gx_glob, own in ((0, self.eb * self.P, True), (1, self.ee * self.P, self.own_right)):
            if not own:
                continue
            dmask = (c_gy == 0) | (c_gy == NY - 1) | (gx_glob == 0) | (gx_glob == t.NXg - 1)
            idx = torch.as_tensor(side * m + np.nonzero(dmask)[0], device=self.device)
            R[idx, idx] = 1.0
        return R.view(2, m, 2, m).permute(0, 2, 1, 3).contiguous()

    def _between(self, W, B):
        if self.G == 1:
            return
        h = torch.stack((W[0], W[-1] if self.own_right else W[-1] - B[-1]))
        xb2 = self._reduced_solve(h)
        W[0] = xb2[:self.m]
        W[-1] = xb2[self.m:]
