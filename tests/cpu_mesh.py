"""Test helper (not a test module): a CPU stand-in for sem_amd.device.Mesh on an element-column
strip, with the fused descriptor semantics of sem_apply (include/sem_ops.h) computed by the oracle.

Used where no GPU exists (the gloo tests of the partitioned solver): only local elements
contribute to the strip's partial sums, the Dirichlet rows of an interface line are written by its
right-hand owner, and a position range writes only the output lines of those element positions
-- the documented semantics of the HIP kernels."""
import numpy as np
import torch


class CPUStripMesh:
    def __init__(self, P, nex, ney, dx, dy, ex_begin=0, ex_end=None):
        ex_end = nex if ex_end is None else ex_end
        self.P, self.nex, self.ney, self.dx, self.dy = P, nex, ney, dx, dy
        self.ex_begin, self.ex_end = ex_begin, ex_end
        self.NX, self.NY = nex * P + 1, ney * P + 1
        self.N = self.NX * self.NY
        self.line_begin, self.line_end = ex_begin * P, ex_end * P
        self.n_local = (self.line_end - self.line_begin + 1) * self.NY
        self.dof_begin = self.line_begin * self.NY
        self.device = torch.device("cpu")
        self.launches = []

    def to_device(self, v, dtype=torch.float64):
        t = v.to(dtype=dtype) if isinstance(v, torch.Tensor) else torch.as_tensor(np.ascontiguousarray(v), dtype=dtype)
        return t.contiguous()

    @staticmethod
    def _np(t):
        return None if t is None else t.numpy()

    def apply(self, x, y=None, *, c_mass=0.0, c_stiff=0.0, c_gradx=0.0, c_grady=0.0, cu=None, cv=None, c_extra=0.0,
              ea=None, eb=None, ec=None, ed=None, c_acc=0.0, dir_mode=0, dir_mask=None, dir_val=None, dir_sides=0,
              algo=0, pos=None, stream=None):
        from oracle import sem_oracle as O
        self.launches.append(pos)
        P, NY = self.P, self.NY
        xn = x.numpy()
        z = O.apply_matrix_free(P, self.ex_end - self.ex_begin, self.ney, self.dx, self.dy, xn, c_mass=c_mass,
                                c_stiff=c_stiff, c_gradx=c_gradx, c_grady=c_grady, cu=self._np(cu), cv=self._np(cv))
        idx = np.arange(self.n_local)
        gx, gy = self.line_begin + idx // NY, idx % NY
        own = ~((gx == self.line_end) & (self.ex_end < self.nex))   # pointwise terms: right-hand owner
        if c_extra != 0.0:
            if ea is not None and eb is not None:
                z = z + own * (c_extra * ea.numpy() * eb.numpy())
            if ec is not None and ed is not None:
                z = z + own * (c_extra * ec.numpy() * ed.numpy())
        if y is None:
            y = torch.empty_like(x)
        if c_acc != 0.0:
            z = z + own * (c_acc * y.numpy())
        if dir_mode:
            if dir_mask is not None:
                dm = dir_mask.numpy() != 0
            else:
                dm = (((dir_sides & 1) != 0) & (gx == 0)) | (((dir_sides & 2) != 0) & (gx == self.NX - 1)) | \
                     (((dir_sides & 4) != 0) & (gy == 0)) | (((dir_sides & 8) != 0) & (gy == NY - 1))
            owner = ~((gx == self.line_end) & (self.ex_end < self.nex))
            g = np.zeros(self.n_local) if dir_val is None else dir_val.numpy()
            z = z.copy()
            sel = dm & owner
            z[sel] = (xn[sel] - g[sel]) if dir_mode == 1 else g[sel]
            z[dm & ~owner] = 0.0
        if pos is None:
            write = np.ones(self.n_local, dtype=bool)
        else:
            ncols = self.ex_end - self.ex_begin
            lo, hi = pos
            lines = np.zeros(self.line_end - self.line_begin + 1, dtype=bool)
            for p in range(lo, hi):
                if p < ncols:
                    lines[p * P:p * P + P] = True
                else:
                    lines[ncols * P] = True
            write = lines[idx // NY]
        yn = y.numpy()
        yn[write] = z[write]
        return y

    def _own_dir(self, dir_mask, dir_sides):
        idx = np.arange(self.n_local)
        gx, gy = self.line_begin + idx // self.NY, idx % self.NY
        own = ~((gx == self.line_end) & (self.ex_end < self.nex))
        if dir_mask is not None:
            dm = dir_mask.numpy() != 0
        else:
            dm = (((dir_sides & 1) != 0) & (gx == 0)) | (((dir_sides & 2) != 0) & (gx == self.NX - 1)) | \
                 (((dir_sides & 4) != 0) & (gy == 0)) | (((dir_sides & 8) != 0) & (gy == self.NY - 1))
        return own, dm, gx * self.NY + gy

    def ns_apply(self, u=None, v=None, p=None, ru=None, rv=None, rc=None, *, c_mass=0.0, c_stiff=0.0, c_gradx=0.0,
                 c_grady=0.0, cu=None, cv=None, juu=None, juv=None, jvu=None, jvv=None, c_T=0.0, T=None, c_div=1.0,
                 dval_u=None, dval_v=None, dir_mask=None, dir_sides=0, pin=-1, pin_val=0.0, pin_first=False,
                 stream=None):
        """sem_ns_apply (include/sem_ops.h) on the strip, composed from strip applies: partial sums over
        the strip's elements; pointwise terms, Dirichlet rows and the pin of the right interface line
        left to its right-hand owner."""
        n = self.n_local
        zero = torch.zeros(n, dtype=torch.float64)
        u = zero if u is None else u
        v = zero if v is None else v
        p = zero if p is None else p
        own, dm, gq = self._own_dir(dir_mask, dir_sides)
        sysk = dict(c_mass=c_mass, c_stiff=c_stiff, c_gradx=c_gradx, c_grady=c_grady, cu=cu, cv=cv)
        A = lambda x, **kw: self.apply(x, **kw).numpy()   # noqa: E731
        pt = lambda c, x: own * (c.numpy() * x.numpy()) if c is not None else 0.0   # noqa: E731
        un, vn, pn = u.numpy(), v.numpy(), p.numpy()
        if ru is not None:
            z = A(u, **sysk) + pt(juu, u) + pt(juv, v) + A(p, c_gradx=1.0)
            z[dm] = own[dm] * (un[dm] - (dval_u.numpy()[dm] if dval_u is not None else 0.0))
            ru.copy_(torch.from_numpy(z))
        if rv is not None:
            z = A(v, **sysk) + pt(jvu, u) + pt(jvv, v) + A(p, c_grady=1.0)
            if T is not None:
                z = z + c_T * A(T, c_mass=1.0)
            z[dm] = own[dm] * (vn[dm] - (dval_v.numpy()[dm] if dval_v is not None else 0.0))
            rv.copy_(torch.from_numpy(z))
        if rc is not None:
            z = c_div * (A(u, c_gradx=1.0) + A(v, c_grady=1.0))
            pinned = gq == pin
            pinrow = own * (pn - pin_val)
            if pin_first:
                z[pinned] = pinrow[pinned]
            z[dm] = A(p, c_stiff=1.0)[dm]
            if not pin_first:
                z[pinned] = pinrow[pinned]
            rc.copy_(torch.from_numpy(z))
        return ru, rv, rc

    def condensed_blocks(self, blocks, *, c_mass=0.0, c_stiff=0.0, c_gradx=0.0, c_grady=0.0, cu=None, cv=None,
                         juu=None, juv=None, jvu=None, jvv=None, dir_mask=None, dir_sides=0, ncomp=2, cols=None,
                         stream=None):
        """sem_condensed_blocks (include/sem_ops.h) on the strip, from the oracle's assembled operators: the
        whole-mesh Jacobian built from this strip's coefficient vectors (rows outside the strip unused),
        Dirichlet rows as identity rows, cut to the strip's pieces (tests/velocity_blocks.extract layout),
        the right interface line's own block left to the strip on its right (the two partial blocks of a
        shared line sum to the whole-mesh block, as the kernel's do)."""
        import scipy.sparse as sp
        from oracle import sem_oracle as O
        from velocity_blocks import extract
        from sem_amd.solvers.velocity_solve import VelocityJacobianSolver
        P, nex, ney, dx, dy, N = self.P, self.nex, self.ney, self.dx, self.dy, self.N
        if getattr(self, "_ops", None) is None:
            self._ops = (O.global_mass_matrix(P, nex, ney, dx, dy), O.global_stiffness_matrix(P, nex, ney, dx, dy),
                         *O.global_gradient_matrices(P, nex, ney, dx, dy))
        M, K, Gx, Gy = self._ops
        sl = slice(self.dof_begin, self.dof_begin + self.n_local)

        def glob(t, fill=0.0):
            a = np.full(N, fill)
            if t is not None:
                a[sl] = t.numpy()
            return a

        A = c_mass * M + c_stiff * K + c_gradx * sp.diags(glob(cu, 1.0)) @ Gx + c_grady * sp.diags(glob(cv, 1.0)) @ Gy
        if ncomp == 2:
            J = sp.bmat([[A + sp.diags(glob(juu)), sp.diags(glob(juv))], [sp.diags(glob(jvu)), A + sp.diags(glob(jvv))]])
        else:
            J = A + sp.diags(glob(juu))
        _, dm, gq = self._own_dir(dir_mask, dir_sides)
        dirg = np.zeros(N, dtype=bool)
        dirg[gq[dm]] = True
        mask = np.tile(dirg, ncomp)
        J = J.tolil()
        J[mask, :] = 0
        J[mask, mask] = 1
        pcs = extract(J.toarray(), P, nex, ney, ncomp=ncomp)
        eb, ee = self.ex_begin, self.ex_end
        c0, c1 = (eb, ee) if cols is None else cols
        for k in ("aIB", "aBI", "E", "F"):
            blocks[k].copy_(torch.as_tensor(pcs[k][eb:ee]).reshape(blocks[k].shape))
        D = pcs["D"][eb:ee + 1].copy()
        if ee < nex:
            D[-1] = 0.0
        blocks["D"].copy_(torch.as_tensor(D).reshape(blocks["D"].shape))
        vs = VelocityJacobianSolver(P, ee - eb, ney, "cpu", ncomp=ncomp)
        cond = vs.condense_dense(torch.as_tensor(pcs["AII"][c0:c1]))
        for k, v in cond.items():
            blocks[k].copy_(v.reshape(blocks[k].shape))
        return blocks

    def interface_pack(self, y, bounds, buf, stream=None):
        r = bounds.index(self.ex_begin)
        left, right = (r - 1 if r > 0 else -1), (r if r < len(bounds) - 2 else -1)
        buf.zero_()
        if left >= 0:
            buf[left * self.NY:(left + 1) * self.NY] = y[:self.NY]
        if right >= 0:
            buf[right * self.NY:(right + 1) * self.NY] = y[-self.NY:]

    def interface_unpack(self, buf, bounds, y, stream=None):
        r = bounds.index(self.ex_begin)
        left, right = (r - 1 if r > 0 else -1), (r if r < len(bounds) - 2 else -1)
        if left >= 0:
            y[:self.NY] = buf[left * self.NY:(left + 1) * self.NY]
        if right >= 0:
            y[-self.NY:] = buf[right * self.NY:(right + 1) * self.NY]
