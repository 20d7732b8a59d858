"""World-size 1/2/3/8 gloo tests (CPU) of the element-partitioned velocity solve with nested-dissection strips
(sem_amd/solvers/nested_dissection.py, StripNDSolver): each rank dissects its own element columns -- its element
shares of the oracle's velocity Jacobian (NavierStokes_Solver.py:123-136,176-183) -- down to its Schur complement
on its two interface lines, and the ranks solve the reduced system over the strip-boundary lines together.  The
solution on every rank's lines equals SciPy's sparse solve of the whole Jacobian (the reference's `splu`)."""
import os
import queue
import socket
import time

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch as _torch
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)   # ranks share the host: no BLAS / OpenMP oversubscription
    _torch.set_num_threads(1)
    try:
        import scipy.sparse.linalg as spla
        import torch
        from velocity_blocks import oracle_velocity_jacobian
        from sem_amd.parallel import StripPartition
        from sem_amd.solvers.nested_dissection import StripNDSolver
        P, nex, ney, Re = case
        ref, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
        J = ref.Jvelo
        part = StripPartition(nex, world)
        eb, ee = part.bounds[rank], part.bounds[rank + 1]
        NY, N = ney * P + 1, (nex * P + 1) * (ney * P + 1)
        sl = slice(eb * P * NY, (ee * P + 1) * NY)
        t = lambda a: torch.as_tensor(np.asarray(a)[sl].copy())  # noqa: E731
        kw = dict(c_stiff=1.0, c_gradx=Re, cu=t(u), c_grady=Re, cv=t(v), juu=t(Re * (ref.Gx @ u)),
                  jvv=t(Re * (ref.Gy @ v)), juv=t(Re * (ref.Gy @ u)), jvu=t(Re * (ref.Gx @ v)))
        vs = StripNDSolver(P, nex, ney, "cpu", part.bounds, rank, dist)
        vs.factor_coeffs(1.0 / nex, 1.0 / ney, **kw)
        r = np.random.default_rng(17)
        b = r.uniform(-1, 1, 2 * N)
        want = spla.spsolve(J.tocsc(), b)
        got = vs.solve(torch.as_tensor(b[:N][sl].copy()), torch.as_tensor(b[N:][sl].copy()))
        err = max(np.abs(g.numpy() - want[c * N:(c + 1) * N][sl]).max() for c, g in enumerate(got))
        q.put((rank, err / np.abs(want).max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [
    (1, (4, 3, 2, 300.0)),
    (2, (4, 4, 3, 300.0)),     # two columns per strip
    (2, (3, 2, 4, 100.0)),     # one column per strip: the root is a horizontal cut of a 1 x 4 piece
    (2, (2, 2, 1, 50.0)),      # one element per strip: the root is a leaf
    (3, (4, 7, 2, 700.0)),     # uneven strips (3, 2, 2 columns)
    (8, (3, 11, 3, 300.0)),    # cfg5's world size over 11 columns (2, 2, 2, 1, 1, 1, 1, 1)
])
def test_strip_nd_solver_gloo(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, t0 = {}, time.time()
    while len(res) < world:
        try:
            k, v = q.get(timeout=2)
            res[k] = v
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead and time.time() - t0 < 300, f"rank failed (exit codes {dead})"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, e in res.items():
        assert e < 1e-10, (rank, e)
