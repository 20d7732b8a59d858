"""Matrix-free operator objects returned by the SEM facade.

The reference returns SciPy CSR matrices (Solvers/SEM.py:170-223) and pydata
COO 3-tensors (:226-245); its consumers use `A @ x`, `A + B`, `s * A`,
`A.diagonal()`, `A[mask, :] @ x` (NavierStokes_Solver.py:119,157,209),
`tensordot(C, x, (1|2, 0))` (ConvectionDiffusion_Solver.py:82-83,101-102) and
`.tocsr()` for SciPy-only consumers (bmat/splu, NavierStokes_Solver.py:179-184).
`SEMOperator` keeps every such combination in closed form,

    A = cM M + cK K + diag(cu) G_x + diag(cv) G_y + diag(d)        (on one mesh)

so any sum / scaling of mass, stiffness, gradient and contracted convection
operators is still ONE fused kernel launch (include/sem_ops.h, sem_apply).
"""
import numbers

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib


def _is_scalar(s):
    return isinstance(s, numbers.Number) and not isinstance(s, bool)


class SEMOperator:
    __array_priority__ = 100  # make numpy defer `ndarray @ op` / `scalar * op` to us

    def __init__(self, mesh, cM=0.0, cK=0.0, gx=(), gy=(), dg=()):
        self.mesh = mesh
        self.cM, self.cK = float(cM), float(cK)
        self.gx, self.gy, self.dg = tuple(gx), tuple(gy), tuple(dg)
        self.shape = (mesh.n_local, mesh.n_local)
        self.dtype = np.dtype(np.float64)
        self._mat = None

    # ------------------------------------------------------------------ algebra
    def _scaled(self, s):
        s = float(s)
        return SEMOperator(self.mesh, s * self.cM, s * self.cK, [(s * c, v) for c, v in self.gx],
                           [(s * c, v) for c, v in self.gy], [(s * c, v) for c, v in self.dg])

    def _plus(self, other, s):
        if _is_scalar(other) and other == 0:
            return self
        if not isinstance(other, SEMOperator):
            return NotImplemented
        if other.mesh is not self.mesh:
            raise ValueError("operators live on different meshes")
        o = other._scaled(s)
        return SEMOperator(self.mesh, self.cM + o.cM, self.cK + o.cK, self.gx + o.gx, self.gy + o.gy,
                           self.dg + o.dg)

    def __add__(self, other):
        return self._plus(other, 1.0)

    __radd__ = __add__

    def __sub__(self, other):
        return self._plus(other, -1.0)

    def __rsub__(self, other):
        return (-self)._plus(other, 1.0)

    def __neg__(self):
        return self._scaled(-1.0)

    def __mul__(self, s):
        return self._scaled(s) if _is_scalar(s) else NotImplemented

    __rmul__ = __mul__

    def __truediv__(self, s):
        return self._scaled(1.0 / s) if _is_scalar(s) else NotImplemented

    # ------------------------------------------------------------------ materialised coefficients
    def _coeffs(self):
        """Collapse the term lists into the kernel's (cX, cu, cY, cv, d) -- computed once."""
        if self._mat is None:
            def fold(terms):
                if not terms:
                    return 0.0, None
                if all(v is None for _, v in terms):
                    return sum(c for c, _ in terms), None
                acc = torch.zeros(self.mesh.n_local, dtype=torch.float64, device=self.mesh.device)
                for c, v in terms:
                    acc += c if v is None else c * v
                return 1.0, acc

            cX, cu = fold(self.gx)
            cY, cv = fold(self.gy)
            d = None
            if self.dg:
                d = torch.zeros(self.mesh.n_local, dtype=torch.float64, device=self.mesh.device)
                for c, v in self.dg:
                    d += c * v
            self._mat = (cX, cu, cY, cv, d)
        return self._mat

    def apply(self, x, y=None, **kw):
        """Device apply: x, y float64 tensors on the mesh device; kw = Dirichlet / accumulate
        options of Mesh.apply.  Returns y."""
        cX, cu, cY, cv, d = self._coeffs()
        return self.mesh.apply(x, y, c_mass=self.cM, c_stiff=self.cK, c_gradx=cX, cu=cu, c_grady=cY, cv=cv,
                               c_extra=1.0 if d is not None else 0.0, ea=d, eb=x if d is not None else None, **kw)

    def __matmul__(self, x):
        if isinstance(x, torch.Tensor):
            if x.dim() != 1:
                return NotImplemented
            return self.apply(self.mesh.to_device(x))
        x = np.asarray(x)
        if x.ndim != 1:
            return NotImplemented
        if x.shape[0] != self.shape[1]:
            raise ValueError(f"dimension mismatch: operator {self.shape} @ vector {x.shape}")
        return self.apply(self.mesh.to_device(x)).cpu().numpy()

    dot = __matmul__

    def matvec(self, x):
        """SciPy LinearOperator protocol (accepts (N,) or (N, 1))."""
        if isinstance(x, np.ndarray) and x.ndim == 2 and x.shape[1] == 1:
            return (self @ x[:, 0])[:, None]
        return self @ x

    def __getitem__(self, key):
        if isinstance(key, tuple) and len(key) == 2 and key[1] == slice(None):
            return RowRestricted(self, key[0])
        raise TypeError("only row selection A[mask, :] is supported")

    # ------------------------------------------------------------------ host views
    def _tables(self):
        from . import GLL
        P = self.mesh.P
        return GLL.standard_nodes(P)[1], GLL.standard_stiffness_matrix(P), GLL.standard_gradient_matrix(P)

    def _host(self, t):
        return None if t is None else t.detach().cpu().numpy()

    def diagonal(self):
        """Main diagonal (NavierStokes_Solver.py:209 uses M.diagonal())."""
        m = self.mesh
        w, Ks, Gs = self._tables()
        mx, my = m.weights_1d()
        from .device import _assembled_diag
        kx = _assembled_diag(np.diag(Ks), m.P, m.ex_begin, m.ex_end, m.line_begin, m.line_end)
        ky = _assembled_diag(np.diag(Ks), m.P, 0, m.ney, 0, m.NY - 1)
        gxd = _assembled_diag(np.diag(Gs), m.P, m.ex_begin, m.ex_end, m.line_begin, m.line_end)
        gyd = _assembled_diag(np.diag(Gs), m.P, 0, m.ney, 0, m.NY - 1)
        cX, cu, cY, cv, d = self._coeffs()
        out = self.cM * (m.dx / 2) * (m.dy / 2) * np.outer(mx, my).ravel()
        out = out + self.cK * ((m.dy / m.dx) * np.outer(kx, my) + (m.dx / m.dy) * np.outer(mx, ky)).ravel()
        out = out + cX * (1.0 if cu is None else self._host(cu)) * ((m.dy / 2) * np.outer(gxd, my)).ravel()
        out = out + cY * (1.0 if cv is None else self._host(cv)) * ((m.dx / 2) * np.outer(mx, gyd)).ravel()
        if d is not None:
            out = out + self._host(d)
        return out

    def tocsr(self):
        """Materialise as SciPy CSR for SciPy-only consumers (bmat / splu).  Not used by any
        apply.  Built like SEM.assemble (SEM.py:113-146): the nonzero element entries of every
        term as unsummed (row, col, value) triplets, summed by one COO->CSR conversion, so the
        sparsity pattern -- including entries that cancel to an explicit 0 -- is the reference's."""
        m = self.mesh
        w, Ks, Gs = self._tables()
        P, NY = m.P, m.NY
        xr = (m.ex_begin, m.ex_end, m.line_begin)
        yr = (0, m.ney, 0)
        W = np.diag(w)
        cX, cu, cY, cv, d = self._coeffs()
        terms = []  # (coef, x-table, x-scale, y-table, y-scale, row weights)
        if self.cM:
            terms.append((self.cM, W, m.dx / 2, W, m.dy / 2, None))
        if self.cK:
            terms.append((self.cK, Ks, 2 / m.dx, W, m.dy / 2, None))
            terms.append((self.cK, W, m.dx / 2, Ks, 2 / m.dy, None))
        if cX:
            terms.append((cX, Gs, 1.0, W, m.dy / 2, cu))
        if cY:
            terms.append((cY, W, m.dx / 2, Gs, 1.0, cv))
        R, Cc, V = [], [], []
        for coef, tx, sx, ty, sy, rw in terms:
            ar, ac, av = _element_triplets(sx * tx, P, *xr)
            br, bc, bv = _element_triplets(sy * ty, P, *yr)
            rows = (ar[:, None] * NY + br[None, :]).ravel()
            cols = (ac[:, None] * NY + bc[None, :]).ravel()
            vals = coef * (av[:, None] * bv[None, :]).ravel()
            if rw is not None:
                vals = vals * self._host(rw)[rows]
            R.append(rows), Cc.append(cols), V.append(vals)
        if d is not None:
            idx = np.arange(self.shape[0])
            R.append(idx), Cc.append(idx), V.append(self._host(d))
        if not R:
            return sp.csr_matrix(self.shape)
        A = sp.coo_matrix((np.concatenate(V), (np.concatenate(R), np.concatenate(Cc))), shape=self.shape).tocsr()
        A.sum_duplicates()
        return A

    def toarray(self):
        return self.tocsr().toarray()

    def __repr__(self):
        return (f"<SEMOperator {self.shape} P={self.mesh.P} mesh={self.mesh.nex}x{self.mesh.ney} cM={self.cM} "
                f"cK={self.cK} gx_terms={len(self.gx)} gy_terms={len(self.gy)} diag_terms={len(self.dg)}>")


def _element_triplets(table, P, e_lo, e_hi, g_lo):
    """Unsummed 1-D element entries (row, col, value) of `table` over elements [e_lo, e_hi),
    zero table entries dropped as np.nonzero does in SEM.assemble (SEM.py:134)."""
    ii, kk = np.nonzero(table)
    base = np.arange(e_lo, e_hi)[:, None] * P - g_lo
    return (base + ii).ravel(), (base + kk).ravel(), np.tile(table[ii, kk], e_hi - e_lo)


class RowRestricted:
    """`A[mask, :]`: applies A on the device and returns the selected rows."""

    def __init__(self, op, rows):
        self.op, self.rows = op, rows

    def __matmul__(self, x):
        y = self.op @ x
        if isinstance(y, torch.Tensor):
            rows = self.rows if isinstance(self.rows, torch.Tensor) else torch.as_tensor(self.rows, device=y.device)
            return y[rows]
        return y[np.asarray(self.rows)]

    def tocsr(self):
        return self.op.tocsr()[np.asarray(self.rows), :]


class ConvectionTensor:
    """Stand-in for the 8-D-assembled 3-tensor C_x / C_y (SEM.py:226-245).  Only its
    contractions with a vector are ever used by consumers; both have closed forms:
        tensordot(C_x, u, (1,0)) = diag(u) G_x          (ConvectionDiffusion_Solver.py:82-83)
        tensordot(C_x, T, (2,0)) = diag(G_x T)          (ConvectionDiffusion_Solver.py:101-102)
    """

    def __init__(self, mesh, axis):
        if axis not in ("x", "y"):
            raise ValueError("axis must be 'x' or 'y'")
        self.mesh, self.axis = mesh, axis
        self.shape = (mesh.n_local,) * 3

    def contract(self, vec, axis):
        m = self.mesh
        v = m.to_device(vec)
        if v.numel() != m.n_local:
            raise ValueError("vector length does not match the mesh")
        if axis == 1:
            return SEMOperator(m, gx=[(1.0, v)]) if self.axis == "x" else SEMOperator(m, gy=[(1.0, v)])
        if axis == 2:
            g = m.apply(v, c_gradx=1.0) if self.axis == "x" else m.apply(v, c_grady=1.0)
            return SEMOperator(m, dg=[(1.0, g)])
        raise ValueError("contraction axis must be 1 or 2")


class COO3:
    """Sparse 3-tensor in coordinate form: what SEM.assemble returns for an 8-D element array
    (SEM.py:139-145, a pydata-sparse `COO(coords, data, shape)`).  A host-side format for consumers
    that assemble their own 3-tensors; the convection operators of global_convection_matrices stay
    matrix-free (ConvectionTensor).  Duplicate coordinates are kept and summed by every operation,
    as pydata-sparse does."""

    def __init__(self, coords, data, shape):
        self.coords = np.asarray(coords, dtype=np.int64)
        self.data = np.asarray(data, dtype=np.float64)
        self.shape = tuple(int(d) for d in shape)
        self.ndim = len(self.shape)

    @property
    def nnz(self):
        return self.data.size

    def contract(self, vec, axis):
        """tensordot(self, vec, (axis, 0)): the 2-tensor over the remaining axes, as SciPy CSR
        (coordinates summed in entry order, as pydata-sparse's COO -> CSR)."""
        x = vec.detach().cpu().numpy() if isinstance(vec, torch.Tensor) else np.asarray(vec, dtype=np.float64)
        if x.ndim != 1 or x.shape[0] != self.shape[axis]:
            raise ValueError("vector length does not match the contracted axis")
        keep = [d for d in range(3) if d != axis]
        data = self.data * x[self.coords[axis]]
        return sp.coo_matrix((data, (self.coords[keep[0]], self.coords[keep[1]])),
                             shape=(self.shape[keep[0]], self.shape[keep[1]])).tocsr()

    def todense(self):
        out = np.zeros(self.shape)
        np.add.at(out, tuple(self.coords), self.data)
        return out


def tensordot(a, b, axes, return_type=None):
    """pydata-sparse `tensordot(C, x, (1|2, 0), return_type=...)` for the convection tensors
    (matrix-free ConvectionTensor -> SEMOperator) and for assembled COO3 tensors (-> SciPy CSR)."""
    del return_type
    if isinstance(a, (ConvectionTensor, COO3)):
        ax, bx = axes
        if bx != 0:
            raise ValueError("only contraction with a vector's axis 0 is supported")
        if isinstance(a, COO3) and ax not in (0, 1, 2):
            raise ValueError("contraction axis must be 0, 1 or 2")
        return a.contract(b, ax)
    raise TypeError("tensordot is provided for ConvectionTensor and COO3 operands")


# device-side Dirichlet helpers re-exported for solver counterparts
DIR_NONE, DIR_IDENTITY, DIR_REPLACE = _lib.DIR_NONE, _lib.DIR_IDENTITY, _lib.DIR_REPLACE
