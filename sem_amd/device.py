"""Device-side mesh handle: owns one libsemops handle and launches the kernels.

PyTorch-ROCm is plumbing here: it provides device buffers, the current HIP
stream and (for multi-GPU) torch.distributed/RCCL.  All arithmetic of the
operator layer runs in the HIP kernels of libsemops.
"""
import contextlib
import ctypes as C
import gc

import numpy as np
import torch

from . import _lib


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("the SEM operator layer runs on a ROCm GPU (gfx950); no GPU is visible -- "
                           "there is no CPU fallback")


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class Mesh:
    """N_ex x N_ey elements of order P with widths dx, dy, holding element columns
    [ex_begin, ex_end) on one GPU (the whole mesh by default)."""

    def __init__(self, P, nex, ney, dx, dy, ex_begin=0, ex_end=None, device=None):
        require_gpu()
        lib = _lib.load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
        ex_end = nex if ex_end is None else ex_end
        h = C.c_void_p()
        _lib.check(lib.sem_create(int(P), int(nex), int(ney), float(dx), float(dy), int(ex_begin), int(ex_end),
                                  self.device.index, C.byref(h)))
        self._h = h
        self._lib = lib
        info = _lib.SemInfo()
        _lib.check(lib.sem_get_info(h, C.byref(info)))
        self.P, self.nex, self.ney = info.P, info.nex, info.ney
        self.dx, self.dy = info.dx, info.dy
        self.ex_begin, self.ex_end = info.ex_begin, info.ex_end
        self.NX, self.NY, self.N = info.NX, info.NY, info.N
        self.line_begin, self.line_end = info.line_begin, info.line_end
        self.n_local, self.dof_begin = info.n_local, info.dof_begin

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.sem_destroy(h)
            self._h = None

    @property
    def key(self):
        return (self.P, self.nex, self.ney, self.dx, self.dy, self.ex_begin, self.ex_end, self.device.index)

    # ------------------------------------------------------------------ helpers
    def to_device(self, v, dtype=torch.float64):
        if isinstance(v, torch.Tensor):
            t = v.to(device=self.device, dtype=dtype)
        else:
            t = torch.as_tensor(np.ascontiguousarray(v), dtype=dtype, device=self.device)
        return t.contiguous()

    def _vec(self, t, name):
        if t is None:
            return None
        if not isinstance(t, torch.Tensor) or t.device != self.device or t.dtype != torch.float64:
            raise ValueError(f"{name} must be a float64 tensor on {self.device}")
        if not t.is_contiguous() or t.numel() != self.n_local:
            raise ValueError(f"{name} must be contiguous with {self.n_local} entries, got {tuple(t.shape)}")
        return t

    def stream_ptr(self, stream=None):
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        return C.c_void_p(s.cuda_stream)

    # ------------------------------------------------------------------ kernels
    def apply(self, x, y=None, *, c_mass=0.0, c_stiff=0.0, c_gradx=0.0, c_grady=0.0, cu=None, cv=None, c_extra=0.0,
              ea=None, eb=None, ec=None, ed=None, c_acc=0.0, dir_mode=_lib.DIR_NONE, dir_mask=None, dir_val=None,
              dir_sides=0, algo=_lib.ALGO_AUTO, pos=None, stream=None):
        """Fused operator apply (include/sem_ops.h, sem_apply).  pos = (begin, end): write only the
        output lines of those element positions of the strip (0..ncols, ncols = closing line)."""
        x = self._vec(x, "x")
        if y is None:
            y = torch.empty_like(x)
        self._vec(y, "y")
        for nm, t in (("cu", cu), ("cv", cv), ("ea", ea), ("eb", eb), ("ec", ec), ("ed", ed), ("dir_val", dir_val)):
            self._vec(t, nm)
        if dir_mask is not None:
            if dir_mask.dtype != torch.uint8 or dir_mask.device != self.device or dir_mask.numel() != self.n_local:
                raise ValueError("dir_mask must be a uint8 tensor of n_local entries on the mesh device")
        d = _lib.SemApplyDesc(float(c_mass), float(c_stiff), float(c_gradx), float(c_grady), _ptr(cu), _ptr(cv),
                              float(c_extra), _ptr(ea), _ptr(eb), _ptr(ec), _ptr(ed), float(c_acc), int(dir_mode),
                              _ptr(dir_mask), _ptr(dir_val), int(dir_sides), int(algo),
                              *((0, 0) if pos is None else (int(pos[0]), int(pos[1]))))
        _lib.check(self._lib.sem_apply(self._h, C.byref(d), _ptr(x), _ptr(y), self.stream_ptr(stream)))
        return y

    def kernel_name(self, algo=_lib.ALGO_AUTO):
        buf = C.create_string_buffer(128)
        _lib.check(self._lib.sem_kernel_name(self._h, int(algo), buf, 128))
        return buf.value.decode()

    def gather_elements(self, u, out=None, stream=None):
        """SEM.scatter (SEM.py:149-167) on the device: u[N] -> u_e[m, n, i, j]."""
        u = self._vec(u, "u")
        n = self.P + 1
        shape = (self.ex_end - self.ex_begin, self.ney, n, n)
        out = torch.empty(shape, dtype=torch.float64, device=self.device) if out is None else out
        if out.shape != shape or not out.is_contiguous() or out.dtype != torch.float64:
            raise ValueError(f"out must be a contiguous float64 tensor of shape {shape}")
        _lib.check(self._lib.sem_gather_elements(self._h, _ptr(u), _ptr(out), self.stream_ptr(stream)))
        return out

    def dss(self, a_e, out=None, stream=None):
        """SEM.assemble for a 4-D element array (SEM.py:113-127): direct-stiffness summation."""
        n = self.P + 1
        shape = (self.ex_end - self.ex_begin, self.ney, n, n)
        if tuple(a_e.shape) != shape:
            raise ValueError(f"element array must have shape {shape}, got {tuple(a_e.shape)}")
        a_e = self.to_device(a_e)
        out = torch.empty(self.n_local, dtype=torch.float64, device=self.device) if out is None else self._vec(out,
                                                                                                             "out")
        _lib.check(self._lib.sem_dss(self._h, _ptr(a_e), _ptr(out), self.stream_ptr(stream)))
        return out

    def interface_pack(self, y, bounds, buf, stream=None):
        b = (C.c_int * len(bounds))(*bounds)
        _lib.check(self._lib.sem_interface_pack(self._h, _ptr(y), b, len(bounds) - 1, _ptr(buf),
                                                self.stream_ptr(stream)))

    def interface_unpack(self, buf, bounds, y, stream=None):
        b = (C.c_int * len(bounds))(*bounds)
        _lib.check(self._lib.sem_interface_unpack(self._h, _ptr(buf), b, len(bounds) - 1, _ptr(y),
                                                  self.stream_ptr(stream)))

    def velocity_blocks(self, blocks, *, c_mass=0.0, c_stiff=0.0, c_gradx=0.0, c_grady=0.0, cu=None, cv=None,
                        juu=None, juv=None, jvu=None, jvv=None, dir_mask=None, dir_sides=0, ncomp=2, cols=None,
                        stream=None):
        """Static-condensation pieces of the NS velocity Jacobian (include/sem_ops.h,
        sem_velocity_blocks) into `blocks` (VelocityJacobianSolver.empty_blocks layout); ncomp=1:
        the scalar operator A + diag(juu) alone.  cols=(c0, c1): blocks["AII"] holds the dense
        interiors of element columns [c0, c1) only."""
        for nm, t in (("cu", cu), ("cv", cv), ("juu", juu), ("juv", juv), ("jvu", jvu), ("jvv", jvv)):
            self._vec(t, nm)
        if dir_mask is not None and (dir_mask.dtype != torch.uint8 or dir_mask.numel() != self.n_local):
            raise ValueError("dir_mask must be a uint8 tensor of n_local entries")
        sizes = (C.c_int64 * 6)()
        _lib.check(self._lib.sem_line_block_sizes(self._h, int(ncomp), sizes))
        names = ("AII", "D", "aIB", "aBI", "E", "F")
        c0, c1 = (self.ex_begin, self.ex_end) if cols is None else (int(cols[0]), int(cols[1]))
        if not self.ex_begin <= c0 < c1 <= self.ex_end:
            raise ValueError("cols must be a non-empty element-column range of the handle's strip")
        sizes[0] = sizes[0] // (self.ex_end - self.ex_begin) * (c1 - c0)
        for nm, sz in zip(names, sizes):
            t = blocks.get(nm)
            if sz and (t is None or t.numel() != sz or t.dtype != torch.float64 or t.device != self.device
                       or not t.is_contiguous()):
                raise ValueError(f"block {nm} must be a contiguous float64 tensor of {sz} entries on {self.device}")
        d = _lib.SemVelocityDesc(float(c_mass), float(c_stiff), float(c_gradx), float(c_grady), _ptr(cu), _ptr(cv),
                                 _ptr(juu), _ptr(juv), _ptr(jvu), _ptr(jvv), _ptr(dir_mask), int(dir_sides),
                                 int(ncomp), c0, c1)
        _lib.check(self._lib.sem_velocity_blocks(self._h, C.byref(d), *(_ptr(blocks.get(nm)) for nm in names),
                                                 self.stream_ptr(stream)))
        return blocks

    def condensed_blocks(self, blocks, *, c_mass=0.0, c_stiff=0.0, c_gradx=0.0, c_grady=0.0, cu=None, cv=None,
                         juu=None, juv=None, jvu=None, jvv=None, dir_mask=None, dir_sides=0, ncomp=2, cols=None,
                         stream=None):
        """The velocity (ncomp=2) or scalar (ncomp=1) Jacobian in the nested condensation's layout
        (include/sem_ops.h, sem_condensed_blocks, ABI 7): blocks["Aii", "Aie", "Aei", "Aed", "Aeu", "Ael"]
        hold element columns cols = (c0, c1); "D", "aIB", "aBI", "E", "F" the whole mesh's interface pieces."""
        for nm, t in (("cu", cu), ("cv", cv), ("juu", juu), ("juv", juv), ("jvu", jvu), ("jvv", jvv)):
            self._vec(t, nm)
        if dir_mask is not None and (dir_mask.dtype != torch.uint8 or dir_mask.numel() != self.n_local):
            raise ValueError("dir_mask must be a uint8 tensor of n_local entries")
        c0, c1 = (self.ex_begin, self.ex_end) if cols is None else (int(cols[0]), int(cols[1]))
        if not self.ex_begin <= c0 < c1 <= self.ex_end:
            raise ValueError("cols must be a non-empty element-column range of the handle's strip")
        line = (C.c_int64 * 6)()
        _lib.check(self._lib.sem_line_block_sizes(self._h, int(ncomp), line))
        cs = (C.c_int64 * 6)()
        _lib.check(self._lib.sem_condensed_block_sizes(self._h, int(ncomp), cs))
        cnames = ("Aii", "Aie", "Aei", "Aed", "Aeu", "Ael")
        lnames = ("D", "aIB", "aBI", "E", "F")
        want = [(nm, cs[i] * (c1 - c0)) for i, nm in enumerate(cnames)] + list(zip(lnames, list(line)[1:]))
        for nm, sz in want:
            t = blocks.get(nm)
            if t is None or t.numel() != sz or t.dtype != torch.float64 or t.device != self.device \
                    or not t.is_contiguous():
                raise ValueError(f"block {nm} must be a contiguous float64 tensor of {sz} entries on {self.device}")
        d = _lib.SemVelocityDesc(float(c_mass), float(c_stiff), float(c_gradx), float(c_grady), _ptr(cu), _ptr(cv),
                                 _ptr(juu), _ptr(juv), _ptr(jvu), _ptr(jvv), _ptr(dir_mask), int(dir_sides),
                                 int(ncomp), c0, c1)
        _lib.check(self._lib.sem_condensed_blocks(self._h, C.byref(d), *(_ptr(blocks[nm]) for nm in cnames + lnames),
                                                  self.stream_ptr(stream)))
        return blocks

    def _line_view(self, t, name):
        """u, v, ru, rv of sem_ns_apply: a plain vector, or an (NX, NY) view with row stride >= NY."""
        if t is None:
            return None, 0
        if t.dim() == 1:
            return self._vec(t, name), 0
        if (not isinstance(t, torch.Tensor) or t.device != self.device or t.dtype != torch.float64
                or tuple(t.shape) != (self.NX, self.NY) or t.stride(1) != 1 or t.stride(0) < self.NY):
            raise ValueError(f"{name} must be a float64 ({self.NX}, {self.NY}) line view on {self.device}")
        return t, t.stride(0)

    def ns_apply(self, u=None, v=None, p=None, ru=None, rv=None, rc=None, *, c_mass=0.0, c_stiff=0.0, c_gradx=0.0,
                 c_grady=0.0, cu=None, cv=None, juu=None, juv=None, jvu=None, jvv=None, c_T=0.0, T=None, c_div=1.0,
                 dval_u=None, dval_v=None, dir_mask=None, dir_sides=0, pin=-1, pin_val=0.0, pin_first=False,
                 stream=None):
        """Fused Navier-Stokes residuals (include/sem_ops.h, sem_ns_apply): ru, rv, rc in one launch.
        u, v, ru, rv are plain vectors or (NX, NY) line views sharing one row stride (the velocity
        solve's interleaved [u | v] lines); a None output is not computed."""
        pitch = set()
        views = []
        for nm, t in (("u", u), ("v", v), ("ru", ru), ("rv", rv)):
            t, s = self._line_view(t, nm)
            views.append(t)
            if t is not None:
                pitch.add(s)
        if len(pitch) > 1:
            raise ValueError("u, v, ru, rv must share one layout")
        for nm, t in (("p", p), ("rc", rc), ("T", T), ("cu", cu), ("cv", cv), ("juu", juu), ("juv", juv),
                      ("jvu", jvu), ("jvv", jvv), ("dval_u", dval_u), ("dval_v", dval_v)):
            self._vec(t, nm)
        if dir_mask is not None and (dir_mask.dtype != torch.uint8 or dir_mask.numel() != self.n_local):
            raise ValueError("dir_mask must be a uint8 tensor of n_local entries")
        d = _lib.SemNsDesc(float(c_mass), float(c_stiff), float(c_gradx), float(c_grady), _ptr(cu), _ptr(cv),
                           _ptr(juu), _ptr(juv), _ptr(jvu), _ptr(jvv), float(c_T), _ptr(T), float(c_div),
                           _ptr(dval_u), _ptr(dval_v), _ptr(dir_mask), int(dir_sides), int(bool(pin_first)), int(pin),
                           float(pin_val), pitch.pop() if pitch else 0)
        _lib.check(self._lib.sem_ns_apply(self._h, C.byref(d), *(_ptr(t) for t in views[:2]), _ptr(p),
                                          *(_ptr(t) for t in views[2:]), _ptr(rc), self.stream_ptr(stream)))
        return views[2], views[3], rc

    # ------------------------------------------------------------------ host-side 1-D tables
    def weights_1d(self):
        """Assembled 1-D GLL weights over the locally held lines (x) and all columns (y)."""
        from . import GLL
        w = GLL.standard_nodes(self.P)[1]
        return (_assembled_diag(w, self.P, self.ex_begin, self.ex_end, self.line_begin, self.line_end),
                _assembled_diag(w, self.P, 0, self.ney, 0, self.NY - 1))


def _assembled_diag(vals, P, e_lo, e_hi, g_lo, g_hi):
    """sum over elements e in [e_lo, e_hi) of vals[local index] at each 1-D node g in [g_lo, g_hi]."""
    out = np.zeros(g_hi - g_lo + 1)
    for e in range(e_lo, e_hi):
        out[e * P - g_lo: e * P + P + 1 - g_lo] += vals
    return out


_MESHES = {}


def get_mesh(P, nex, ney, dx, dy, ex_begin=0, ex_end=None, device=None):
    """Cached Mesh per (P, N_ex, N_ey, dx, dy, partition, device)."""
    require_gpu()
    dev = torch.cuda.current_device() if device is None else int(device)
    ex_end = nex if ex_end is None else ex_end
    key = (int(P), int(nex), int(ney), float(dx), float(dy), int(ex_begin), int(ex_end), dev)
    m = _MESHES.get(key)
    if m is None:
        m = _MESHES[key] = Mesh(P, nex, ney, dx, dy, ex_begin, ex_end, dev)
    return m


@contextlib.contextmanager
def no_gc():
    """Keep Python's cyclic GC from running inside a stream capture: a collection there can run the
    finaliser of an unrelated object (an old hipGraph, a mesh handle) whose device calls are illegal
    while the stream captures, which aborts the process.  torch.cuda.graph collects on entry (an
    explicit gc.collect runs while the GC is disabled); enter no_gc() first so that the capture has
    ended before collection is enabled again: `with no_gc(), torch.cuda.graph(g): ...`."""
    enabled = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if enabled:
            gc.enable()
