"""World-size-2 gloo test (CPU) of the element-strip decomposition and the interface
exchange protocols of sem_amd.parallel (InterfaceExchange: one all-reduce;
NeighborExchange: point-to-point with the two neighbouring strips).

The device kernels cannot run here, so each rank's local apply is the oracle's
matrix-free apply on its own strip of elements (the same partial sums the kernel
forms: only local elements contribute, Dirichlet rows of an interface line are
written by its right-hand owner), and the pack/unpack kernels are replaced by a
CPU test double with their documented slot semantics.  The product's partition,
slot assignment and all-reduce protocol run unchanged."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class StripDouble:
    """CPU stand-in for sem_amd.device.Mesh with the kernels' partition semantics."""

    def __init__(self, P, nex, ney, dx, dy, eb, ee):
        self.P, self.nex, self.ney, self.dx, self.dy, self.eb, self.ee = P, nex, ney, dx, dy, eb, ee
        self.NY = ney * P + 1
        self.line_begin, self.line_end = eb * P, ee * P
        self.n_local = (self.line_end - self.line_begin + 1) * self.NY
        self.dof_begin = self.line_begin * self.NY
        self.device = torch.device("cpu")

    def apply(self, x, sides_mask_global, g):
        from oracle import sem_oracle as O
        y = O.apply_matrix_free(self.P, self.ee - self.eb, self.ney, self.dx, self.dy, x, c_stiff=1.0)
        lines = np.arange(self.line_begin, self.line_end + 1).repeat(self.NY)
        m = sides_mask_global[self.dof_begin:self.dof_begin + self.n_local]
        owner = ~((lines == self.line_end) & (self.ee < self.nex))
        y[m & owner] = x[m & owner] - g[m & owner]
        y[m & ~owner] = 0.0
        return torch.from_numpy(y)

    def interface_pack(self, y, bounds, buf):
        r = bounds.index(self.eb)
        left, right = (r - 1 if r > 0 else -1), (r if r < len(bounds) - 2 else -1)
        buf.zero_()
        if left >= 0:
            buf[left * self.NY:(left + 1) * self.NY] = y[:self.NY]
        if right >= 0:
            buf[right * self.NY:(right + 1) * self.NY] = y[-self.NY:]

    def interface_unpack(self, buf, bounds, y):
        r = bounds.index(self.eb)
        left, right = (r - 1 if r > 0 else -1), (r if r < len(bounds) - 2 else -1)
        if left >= 0:
            y[:self.NY] = buf[left * self.NY:(left + 1) * self.NY]
        if right >= 0:
            y[-self.NY:] = buf[right * self.NY:(right + 1) * self.NY]


def _worker(rank, world, port, P, nex, ney, q, kind="allreduce"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch as _torch
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)   # ranks share the host: no BLAS / OpenMP oversubscription
    _torch.set_num_threads(1)
    try:
        from oracle import sem_oracle as O
        from sem_amd.parallel import StripPartition
        dx, dy = 1.0 / nex, 1.0 / ney
        N = (nex * P + 1) * (ney * P + 1)
        x = np.random.default_rng(3).uniform(-1, 1, N)
        g = np.random.default_rng(4).uniform(-1, 1, N)
        NX, NY = nex * P + 1, ney * P + 1
        gx = np.arange(N) // NY
        mask = (gx == 0) | (gx == NX - 1)
        part = StripPartition(nex, world)
        eb, ee = part.local_range(rank)
        mesh = StripDouble(P, nex, ney, dx, dy, eb, ee)
        sl = slice(mesh.dof_begin, mesh.dof_begin + mesh.n_local)
        y = mesh.apply(x[sl], mask, g[sl])
        y = part.exchanger(mesh, dist, kind=kind)(y)
        want = O.apply_matrix_free(P, nex, ney, dx, dy, x, c_stiff=1.0)
        want[mask] = x[mask] - g[mask]
        err = np.abs(y.numpy() - want[sl]).max() / np.abs(want).max()
        q.put((rank, float(err)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind", ["allreduce", "p2p"])
@pytest.mark.parametrize("world,P,nex,ney", [(2, 4, 6, 5), (2, 8, 9, 4), (3, 5, 7, 3), (4, 3, 8, 2)])
def test_interface_exchange_gloo(world, P, nex, ney, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, nex, ney, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(e < 1e-13 for e in res.values()), res


def test_partition_bounds():
    from sem_amd.parallel import StripPartition
    p = StripPartition(10, 3)
    assert p.bounds == [0, 4, 7, 10]
    assert [p.slots(r) for r in range(3)] == [(-1, 0), (0, 1), (1, -1)]
    with pytest.raises(ValueError):
        StripPartition(2, 3)
    with pytest.raises(ValueError):
        p.exchanger(None, None, kind="ring")


def _worker_gmres(rank, world, port, P, nex, ney, q, kind):
    """Partitioned GMRES: strip matvec + interface exchange, DistributedInner dot products."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch as _torch
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)   # ranks share the host: no BLAS / OpenMP oversubscription
    _torch.set_num_threads(1)
    try:
        from sem_amd.krylov import gmres
        from sem_amd.parallel import DistributedInner, StripPartition
        dx, dy = 1.0 / nex, 1.0 / ney
        N = (nex * P + 1) * (ney * P + 1)
        NX, NY = nex * P + 1, ney * P + 1
        gx = np.arange(N) // NY
        mask = (gx == 0) | (gx == NX - 1)
        b = np.random.default_rng(7).uniform(-1, 1, N)
        part = StripPartition(nex, world)
        eb, ee = part.local_range(rank)
        mesh = StripDouble(P, nex, ney, dx, dy, eb, ee)
        sl = slice(mesh.dof_begin, mesh.dof_begin + mesh.n_local)
        exch = part.exchanger(mesh, dist, kind=kind)
        zero = np.zeros(N)

        def mv(v):
            return exch(mesh.apply(v.numpy(), mask, zero[sl]))

        res = gmres(mv, torch.from_numpy(b[sl].copy()), atol=1e-10, restart=40, maxiter=4000,
                    inner=DistributedInner(part, mesh, dist))
        q.put((rank, res.info, res.iters, res.x.numpy().tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["allreduce", "p2p"])
@pytest.mark.parametrize("world,P,nex,ney", [(2, 4, 6, 4), (3, 3, 7, 3)])
def test_partitioned_gmres_gloo(world, P, nex, ney, kind):
    """A strip-partitioned GMRES solve of the stiffness system with Dirichlet rows reproduces the
    single-domain solve: same iteration count, same solution to the solver tolerance."""
    from oracle import sem_oracle as O
    from sem_amd.krylov import gmres
    dx, dy = 1.0 / nex, 1.0 / ney
    N = (nex * P + 1) * (ney * P + 1)
    NX, NY = nex * P + 1, ney * P + 1
    gx = np.arange(N) // NY
    mask = (gx == 0) | (gx == NX - 1)
    b = np.random.default_rng(7).uniform(-1, 1, N)

    def mv(v):
        y = O.apply_matrix_free(P, nex, ney, dx, dy, v.numpy(), c_stiff=1.0)
        y[mask] = v.numpy()[mask]
        return torch.from_numpy(y)

    ref = gmres(mv, torch.from_numpy(b), atol=1e-10, restart=40, maxiter=4000)
    assert ref.info == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_gmres, args=(r, world, port, P, nex, ney, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict((r, (info, it, np.array(x))) for r, info, it, x in (q.get(timeout=180) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    part_bounds = __import__("sem_amd.parallel", fromlist=["StripPartition"]).StripPartition(nex, world).bounds
    for r, (info, it, x) in out.items():
        assert info == 0 and abs(it - ref.iters) <= 1, (it, ref.iters)
        d0 = part_bounds[r] * P * NY
        assert np.abs(x - ref.x.numpy()[d0:d0 + len(x)]).max() < 1e-8
