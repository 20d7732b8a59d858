"""Element-strip partition across GPUs and the interface-line exchange.

The reference has no domain decomposition.  Here rank r of G
holds element columns [bounds[r], bounds[r+1]).  In the reference's x-major
numbering (SEM.py:110) those are the contiguous global DOF range of lines
[bounds[r]*P, bounds[r+1]*P]; neighbouring strips share exactly one line of
N_ey*P+1 nodes.  Each rank applies the operator to its own elements (partial
sums on its two interface lines; Dirichlet rows on an interface line are
written by its right-hand owner only), then the interface partial sums are
packed into a (G-1)*NY buffer, summed across ranks with one RCCL all-reduce
over xGMI (torch.distributed backend "nccl" = RCCL on ROCm), and unpacked.  The
payload is tiny (28.7 KB at 64^2 elements per GPU, G = 8) -- a latency-bound
collective; nothing else crosses GPUs.

NeighborExchange is the point-to-point alternative: in the x-major numbering an
interface line is a contiguous slice of the local vector (the first / last NY
entries), so each rank sends its two partial-sum lines straight to its left and
right neighbours (one batch of RCCL send/recv pairs over the xGMI links to those
two GPUs) and adds what it receives.  No pack kernel, 2 x NY x 8 bytes per link
and direction, and no rank waits on a ring through all G ranks.  Both exchanges
give bitwise-identical results (each shared node is the sum of exactly two partial
sums, and a + b == b + a in IEEE arithmetic).
"""
import torch


class StripPartition:
    def __init__(self, nex, world):
        if world < 1 or world > nex:
            raise ValueError("need 1 <= world <= N_ex element columns")
        base, extra = divmod(nex, world)
        self.bounds = [0]
        for r in range(world):
            self.bounds.append(self.bounds[-1] + base + (1 if r < extra else 0))
        self.nex, self.world = nex, world

    def local_range(self, rank):
        return self.bounds[rank], self.bounds[rank + 1]

    def slots(self, rank):
        """(left_slot, right_slot) of this rank's interface lines in the exchange buffer (-1 = none)."""
        return (rank - 1 if rank > 0 else -1), (rank if rank < self.world - 1 else -1)

    def exchanger(self, mesh, dist, group=None, kind="allreduce"):
        """Callable y -> y with the interface partial sums assembled across ranks.
        kind: "allreduce" (one collective over all interface slots) or "p2p" (neighbours only)."""
        if kind == "allreduce":
            return InterfaceExchange(self, mesh, dist, group)
        if kind == "p2p":
            return NeighborExchange(self, mesh, dist, group)
        raise ValueError("exchange kind must be 'allreduce' or 'p2p'")


class InterfaceExchange:
    def __init__(self, part, mesh, dist, group=None):
        self.part, self.mesh, self.dist, self.group = part, mesh, dist, group
        self.buf = torch.empty((part.world - 1) * mesh.NY, dtype=torch.float64, device=mesh.device)

    def start(self, y):
        """Pack the interface partial sums and start the all-reduce (returns its work handle; the
        collective runs on the process group's own stream, concurrently with later launches)."""
        self.mesh.interface_pack(y, self.part.bounds, self.buf)
        return self.dist.all_reduce(self.buf, group=self.group, async_op=True)

    def finish(self, y, work):
        work.wait()
        self.mesh.interface_unpack(self.buf, self.part.bounds, y)
        return y

    def __call__(self, y):
        if self.part.world == 1:
            return y
        return self.finish(y, self.start(y))

    def many(self, ys):
        """Assemble the interface lines of several vectors with ONE collective (the three Navier-Stokes
        residuals): each is packed into its own slice of one buffer."""
        n = self.buf.numel()
        if getattr(self, "_mbuf", None) is None or self._mbuf.numel() < len(ys) * n:
            self._mbuf = torch.empty(len(ys) * n, dtype=torch.float64, device=self.mesh.device)
        for i, y in enumerate(ys):
            self.mesh.interface_pack(y, self.part.bounds, self._mbuf[i * n:(i + 1) * n])
        self.dist.all_reduce(self._mbuf[:len(ys) * n], group=self.group)
        for i, y in enumerate(ys):
            self.mesh.interface_unpack(self._mbuf[i * n:(i + 1) * n], self.part.bounds, y)
        return ys


class NeighborExchange:
    """Interface assembly by point-to-point exchange with the two neighbouring strips."""

    def __init__(self, part, mesh, dist, group=None):
        self.part, self.mesh, self.dist, self.group = part, mesh, dist, group
        self.rank = part.bounds.index(mesh.ex_begin if hasattr(mesh, "ex_begin") else mesh.eb)
        self.NY = mesh.NY
        left, right = part.slots(self.rank)
        self.left = self.rank - 1 if left >= 0 else None
        self.right = self.rank + 1 if right >= 0 else None
        # gloo (the one-GPU rehearsal backend) sends and receives host tensors only: stage through host
        self.host = dist.get_backend(group) == "gloo" and mesh.device.type == "cuda"
        bdev = "cpu" if self.host else mesh.device
        self.recv_l = torch.empty(self.NY, dtype=torch.float64, device=bdev) if self.left is not None else None
        self.recv_r = torch.empty(self.NY, dtype=torch.float64, device=bdev) if self.right is not None else None

    def _peer(self, r):
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def start(self, y):
        NY, d = self.NY, self.dist
        ops = []
        if self.left is not None:
            sl = y[:NY].cpu() if self.host else y[:NY]
            ops.append(d.P2POp(d.isend, sl, self._peer(self.left), self.group))
            ops.append(d.P2POp(d.irecv, self.recv_l, self._peer(self.left), self.group))
        if self.right is not None:
            sr = y[-NY:].cpu() if self.host else y[-NY:]
            ops.append(d.P2POp(d.isend, sr, self._peer(self.right), self.group))
            ops.append(d.P2POp(d.irecv, self.recv_r, self._peer(self.right), self.group))
        return d.batch_isend_irecv(ops) if ops else []

    def finish(self, y, reqs):
        for req in reqs:
            req.wait()
        NY = self.NY
        if self.left is not None:
            y[:NY] += self.recv_l.to(y.device)
        if self.right is not None:
            y[-NY:] += self.recv_r.to(y.device)
        return y

    def __call__(self, y):
        if self.part.world == 1:
            return y
        return self.finish(y, self.start(y))

    def many(self, ys):
        """Several vectors, one after the other (the receive buffers are shared)."""
        for y in ys:
            self(y)
        return ys


class StripApply:
    """One partitioned operator apply with the interface assembly.

    overlap=True: the output lines of the strip's two interface positions (first element column,
    closing line) are computed first (two position-ranged launches, sem_apply_desc.pos_*), their
    exchange is started -- an async RCCL all-reduce (or send/recv) on the process group's stream --
    and the interior positions are computed while it runs; then the step waits and unpacks.  The
    interior launch touches neither interface line, so nothing races with the collective.
    overlap=False: one launch over the strip, then the exchange."""

    def __init__(self, part, mesh, dist, group=None, kind="allreduce", overlap=True):
        self.part, self.mesh, self.dist = part, mesh, dist
        self.exch = part.exchanger(mesh, dist, group=group, kind=kind) if part.world > 1 else None
        self.overlap = overlap and self.exch is not None
        self.ncols = mesh.ex_end - mesh.ex_begin

    def __call__(self, x, y=None, **kw):
        m = self.mesh
        if y is None:
            y = torch.empty_like(x)
        if self.exch is None:
            return m.apply(x, y, **kw)
        if not self.overlap:
            m.apply(x, y, **kw)
            return self.exch(y)
        n = self.ncols
        m.apply(x, y, pos=(0, 1), **kw)
        m.apply(x, y, pos=(n, n + 1), **kw)
        work = self.exch.start(y)
        if n > 1:
            m.apply(x, y, pos=(1, n), **kw)
        return self.exch.finish(y, work)


class DistributedInner:
    """Inner products of strip-partitioned vectors for sem_amd.krylov.gmres(inner=...).

    A shared interface line is stored on both neighbouring ranks (with equal values after the
    exchange); it is counted once, on the left-hand rank.  The owned entries are contiguous ranges of
    the local vector (`segments`: a rank > 0 skips its first NY entries), so krylov.gmres runs its
    HIP basis sweeps on those ranges directly -- no mask, no temporary -- and sums the per-rank partial
    products with `reduce` (one all-reduce, RCCL over xGMI under "nccl"): one per Arnoldi step for both
    CGS2 coefficient sets and the norm before the update, one for the norm after it.
    Called as inner(A, w) it is the plain k inner products (gmres_left, tests)."""

    def __init__(self, part, mesh, dist, group=None, segments=None, backend_device=None):
        self.dist, self.group = dist, group
        if segments is None:
            rank = part.bounds.index(mesh.ex_begin if hasattr(mesh, "ex_begin") else mesh.eb)
            segments = [(mesh.NY if rank > 0 else 0, mesh.n_local)]
            n, dev = mesh.n_local, mesh.device
        else:
            n, dev = mesh
        self.segments = [(int(a), int(b)) for a, b in segments]
        self.n = n
        self.own = torch.zeros(n, dtype=torch.float64, device=dev)
        for a, b in self.segments:
            self.own[a:b] = 1.0
        if backend_device is None and dist is not None:
            backend_device = ("cuda" if dist.get_backend(group) == "nccl" else "cpu")
        self.bdev = torch.device(backend_device) if backend_device is not None else None
        self.collectives = 0          # all-reduces issued (profiling: tools/strip_profile.py)

    def reduce(self, t):
        """Sum t (a device tensor) over the ranks, in place; returns t.  Under RCCL the collective stays on
        the device (stream-ordered, no host synchronisation); under gloo it is staged through the host."""
        if self.dist is None:
            return t
        self.collectives += 1
        if self.bdev is None or t.device.type == self.bdev.type:
            self.dist.all_reduce(t, group=self.group)
            return t
        tb = t.to(self.bdev)
        self.dist.all_reduce(tb, group=self.group)
        t.copy_(tb)
        return t

    def __call__(self, A, w):
        h = None
        for a, b in self.segments:
            p = A[:, a:b] @ w[a:b]
            h = p if h is None else h + p
        return self.reduce(h)


class Partition:
    """Element-strip partition of one solver across the ranks of `dist` (torch.distributed, RCCL
    under "nccl"): this rank holds element columns part.local_range(rank).  Passed to
    ConvectionDiffusionSolver(partition=...).  mesh_factory(P, nex, ney, dx, dy, eb, ee) builds the
    strip's mesh (default: a libsemops handle on the current device)."""

    def __init__(self, dist, group=None, exchange="allreduce", overlap=True, mesh_factory=None):
        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.exchange, self.overlap = exchange, overlap
        self.mesh_factory = mesh_factory

    def setup(self, P, nex, ney, dx, dy):
        self.part = StripPartition(nex, self.world)
        eb, ee = self.part.local_range(self.rank)
        if self.mesh_factory is not None:
            mesh = self.mesh_factory(P, nex, ney, dx, dy, eb, ee)
        else:
            from .device import get_mesh
            mesh = get_mesh(P, nex, ney, dx, dy, eb, ee)
        self.mesh = mesh
        self.step = StripApply(self.part, mesh, self.dist, self.group, self.exchange, self.overlap)
        self.inner = DistributedInner(self.part, mesh, self.dist, self.group)
        return mesh

    def max_local_dofs(self):
        """The largest strip's DOF count over all ranks (from the bounds, no communication): a Krylov
        restart length sized from it is the same on every rank, so every rank leaves the Arnoldi loop at the
        same iteration and calls the same collectives (uneven strips gave ranks different
        restarts)."""
        b, P, NY = self.part.bounds, self.mesh.P, self.mesh.NY
        return max((b[r + 1] - b[r]) * P + 1 for r in range(self.world)) * NY

    def local(self, v):
        """This rank's slice of a global vector (x-major numbering)."""
        m = self.mesh
        return v[m.dof_begin:m.dof_begin + m.n_local]

    def assemble(self, *ys):
        """Sum the interface lines of strip partial results (one collective for all of them)."""
        ex = self.step.exch
        if ex is not None:
            ex.many(list(ys))
        return ys

    def backend_device(self):
        """Where collective buffers live: the GPU under RCCL ("nccl"), the host under gloo."""
        if self.dist.get_backend(self.group) == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def norm(self, *ys):
        """2-norm of the stacked global vectors from strips (a shared line counted once)."""
        own = self.inner.own
        s = sum((y.square() * own).sum() for y in ys).reshape(1).to(self.backend_device())
        self.dist.all_reduce(s, group=self.group)
        return float(torch.sqrt(s).item())

    def amax(self, *ys):
        m = torch.stack([y.abs().max() for y in ys]).max().reshape(1).to(self.backend_device())
        self.dist.all_reduce(m, op=self.dist.ReduceOp.MAX, group=self.group)
        return float(m.item())

    def broadcast(self, t, src=0):
        """t (a host or device tensor, same shape on every rank) from rank src, on this rank's device."""
        dev = t.device
        b = t.to(self.backend_device())
        self.dist.broadcast(b, src=src if self.group is None else self.dist.get_global_rank(self.group, src),
                            group=self.group)
        return b.to(dev)

    def gather(self, y):
        """Global vector (every rank) from the local strips; shared lines agree after an exchange."""
        m = self.mesh
        full = torch.zeros(m.N, dtype=y.dtype, device=y.device)
        own = y if self.rank == 0 else y[m.NY:]      # a shared line is taken from its left rank
        off = m.dof_begin if self.rank == 0 else m.dof_begin + m.NY
        full[off:off + own.numel()] = own
        self.dist.all_reduce(full, group=self.group)
        return full
