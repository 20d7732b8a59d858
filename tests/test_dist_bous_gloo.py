"""World-size-2 gloo test (CPU) of the parallel Boussinesq coupler
(sem_amd.solvers.boussinesq.ParallelBoussinesqCoupler, the counterpart of
OpenMDAO/Boussinesq_ParallelCoupler.py): CD on rank 0 and NS on rank 1, blocks exchanged with
all-reduces, the coupled Newton-Krylov iteration replicated.  The device solvers cannot run here, so
both ranks use the oracle-backed solver interface (tests/oracle_solvers.py); the sequential coupler
with the same solvers is the reference result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

CFG = dict(Re=1e3, Ra=1e3, Pr=0.71, P=4, ne=3)


def _solvers():
    from oracle_solvers import OracleCD, OracleNS
    Re, Ra, Pr, P, ne = CFG["Re"], CFG["Ra"], CFG["Pr"], CFG["P"], CFG["ne"]
    cd = OracleCD(1.0, 1.0, Re * Pr, P, ne, ne, T_W=0.5, T_E=-0.5, mtol=1e-12)
    ns = OracleNS(1.0, 1.0, Re, Ra / Pr, P, ne, ne, mtol=1e-12, mtol_newton=1e-12)
    return cd, ns


def _worker(rank, port, mode, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    import torch as _torch
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)   # ranks share the host: no BLAS / OpenMP oversubscription
    _torch.set_num_threads(1)
    try:
        from sem_amd.solvers.boussinesq import ParallelBoussinesqCoupler
        cd, ns = _solvers()
        c = ParallelBoussinesqCoupler(1.0, 1.0, CFG["Re"], CFG["Ra"], CFG["Pr"], CFG["P"], CFG["ne"], CFG["ne"],
                                      CFG["P"], CFG["ne"], CFG["ne"], mode=mode, cd=cd, ns=ns, dist=dist)
        T, u, v, p = c.solve()
        q.put((rank, T, u, v, c.iterations, c.calls))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["JNK", "NJ"])
def test_parallel_coupler_matches_sequential(mode):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    cd, ns = _solvers()
    seq = BoussinesqCoupler(1.0, 1.0, CFG["Re"], CFG["Ra"], CFG["Pr"], CFG["P"], CFG["ne"], CFG["ne"], CFG["P"],
                            CFG["ne"], CFG["ne"], mode=mode, cd=cd, ns=ns)
    Ts, us, vs, _ = seq.solve()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict((o[0], o[1:]) for o in (q.get(timeout=600) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T0, u0, v0, it0, calls0 = out[0]
    T1, u1, v1, it1, calls1 = out[1]
    # both ranks hold the same coupled state and took the same path
    assert np.array_equal(T0, T1) and np.array_equal(u0, u1) and it0 == it1
    # the same coupled solution as the sequential coupler (to the nonlinear tolerance)
    for a, b in ((T0, Ts), (u0, us), (v0, vs)):
        assert np.abs(a - b).max() < 1e-7
    # each rank ran only its own block solves
    assert calls0["ns_update"] == 0 and calls1["cd_update"] == 0
    assert calls0["cd_update"] == calls1["ns_update"] > 0 or mode == "JNK" and it0 == 0


def _worker_partitioned(rank, world, port, key, q, cd_update="central"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch as _torch
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)   # ranks share the host: no BLAS / OpenMP oversubscription
    _torch.set_num_threads(1)
    try:
        from conftest import golden
        from cpu_mesh import CPUStripMesh
        from oracle_solvers import OracleCD, OracleNS
        from sem_amd.solvers.boussinesq import partitioned_coupler
        g = golden("bous.npz")
        Pc, nxc, nyc, Pn, nxn, nyn = (int(a) for a in g[key + "_cfg"])
        Re, Ra, Pr = 1e3, 1e3, 0.71
        c = partitioned_coupler(dist, 1.0, 1.0, Re, Ra, Pr, Pc, nxc, nyc, Pn, nxn, nyn, mesh_factory=CPUStripMesh,
                                mode=str(g[key + "_mode"]), cd_update=cd_update)
        c.ns._central_solver = lambda: OracleNS(1.0, 1.0, Re, Ra / Pr, Pn, nxn, nyn, mtol=1e-13, mtol_newton=1e-13)
        c.cd._central_solver = lambda: OracleCD(1.0, 1.0, Re * Pr, Pc, nxc, nyc, T_W=0.5, T_E=-0.5, mtol=1e-13)
        R = c.residuals(g[key + "_x"])
        c.linearize(g[key + "_x"])
        JR = c.jacobian_apply(g[key + "_dx"])
        T, u, v, p = c.solve()
        q.put((rank, R, JR, T, u, v, c.iterations))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,key,cd_update", [(2, "a", "central"), (2, "c", "central"), (2, "a", "distributed")])
def test_element_partitioned_coupler(world, key, cd_update):
    """cfg5's structure at the golden's size: both solvers strip-partitioned over `world` ranks
    (partitioned_coupler), against the reference solver classes driven through the same coupling
    (tests/golden/bous.npz): coupled residual / Jacobian apply to 1e-12, the same Newton count, the
    fields to the nonlinear tolerance."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from conftest import golden
    g = golden("bous.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_partitioned, args=(r, world, port, key, q, cd_update)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, R, JR, T, u, v, iters in out:
        assert np.abs(R - g[key + "_R"]).max() <= 1e-12 * np.abs(g[key + "_R"]).max(), rank
        assert np.abs(JR - g[key + "_JR"]).max() <= 1e-12 * np.abs(g[key + "_JR"]).max(), rank
        assert iters == int(g[key + "_iters"]), (rank, iters)
        for name, a in zip("Tuv", (T, u, v)):
            ref = g[key + "_" + name]
            assert np.abs(a - ref).max() <= 1e-6 * max(np.abs(ref).max(), 1e-3), (rank, name)
