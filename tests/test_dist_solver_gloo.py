"""World-size 2/3 gloo tests (CPU) of the partitioned convection-diffusion solver
(ConvectionDiffusionSolver(partition=...), sem_amd.parallel.Partition / StripApply):

* the overlapped strip apply (interface positions, async exchange, interior positions) equals the
  unpartitioned operator, for both exchange protocols, with and without overlap;
* the reference methods _get_residuals / _calc_jacobians / _get_dresiduals (global NumPy in,
  global NumPy out) match the oracle's (ConvectionDiffusion_Solver.py:73-121);
* the partitioned device-GMRES Newton step (_get_solution, :158-170) matches the oracle's
  LGMRES solution.

The HIP kernels cannot run here: each rank's strip mesh is tests/cpu_mesh.CPUStripMesh (the
kernels' strip / position-range semantics computed by the oracle).  The product's partition,
overlap schedule, exchanges, distributed inner products and solver logic run unchanged."""
import os
import socket

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
        from cpu_mesh import CPUStripMesh
        from oracle import sem_oracle as O
        from sem_amd.parallel import Partition
        from sem_amd.solvers import ConvectionDiffusionSolver
        P, nex, ney, kind, overlap = case
        Pe = 40.0
        part = Partition(dist, exchange=kind, overlap=overlap, mesh_factory=CPUStripMesh)
        cd = ConvectionDiffusionSolver(1.0, 1.0, Pe, P, nex, ney, T_W=0.5, T_E=-0.5, mtol=1e-10, partition=part)
        ref = O.CDOracle(1.0, 1.0, Pe, P, nex, ney, T_W=0.5, T_E=-0.5)
        r = np.random.default_rng(17)
        T, u, v, dT, du, dv = (r.uniform(-1, 1, cd.N) for _ in range(6))
        errs = {}
        res = cd._get_residuals(T, u, v)
        want = ref.residuals(T, u, v)
        errs["res"] = np.abs(res - want).max() / np.abs(want).max()
        cd._calc_jacobians(T)
        ref.calc_jacobians(T)
        dres = cd._get_dresiduals(dT, du, dv)
        want = ref.dresiduals(dT, du, dv)
        errs["dres"] = np.abs(dres - want).max() / np.abs(want).max()
        # the reference example's flow (Examples/ConvectionDiffusion_Example.py:26-27)
        pts = cd.points
        uf, vf = pts[1] - 0.5, 0.5 - pts[0]
        Ts = cd._get_solution(uf, vf)
        Tr = ref.solution(uf, vf, mtol=1e-10)
        errs["solve"] = np.abs(Ts - Tr).max()
        errs["launches"] = len(cd._mesh.launches)
        errs["ranged"] = sum(1 for p in cd._mesh.launches if p is not None)
        q.put((rank, errs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [
    (2, (4, 5, 3, "allreduce", True)),
    (2, (4, 5, 3, "allreduce", False)),
    (2, (3, 4, 4, "p2p", True)),
    (3, (4, 6, 2, "allreduce", True)),
    (3, (2, 3, 5, "p2p", True)),          # one element column per rank: no interior launch
])
def test_partitioned_cd_solver_gloo(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res, t0 = {}, time.time()
    while len(res) < world:     # fail fast when a rank dies instead of waiting out the queue
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
        assert e["res"] < 1e-13 and e["dres"] < 1e-13, (rank, e)
        assert e["solve"] < 1e-7, (rank, e)
        if case[4]:   # overlapped: every apply is split into position-ranged launches
            assert e["ranged"] == e["launches"], (rank, e)
        else:
            assert e["ranged"] == 0, (rank, e)
