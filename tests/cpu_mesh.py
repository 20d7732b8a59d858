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
