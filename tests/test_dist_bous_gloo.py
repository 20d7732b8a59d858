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


W8 = dict(Re=1e3, Ra=1e3, Pr=0.71, P=4, nex=9, ney=3)   # 9 element columns: strips of 2, 1, ..., 1 over 8 ranks


def _w8_solvers():
    from oracle_solvers import OracleCD, OracleNS
    c = W8
    cd = OracleCD(1.0, 1.0, c["Re"] * c["Pr"], c["P"], c["nex"], c["ney"], T_W=0.5, T_E=-0.5, mtol=1e-13)
    ns = OracleNS(1.0, 1.0, c["Re"], c["Ra"] / c["Pr"], c["P"], c["nex"], c["ney"], mtol=1e-13, mtol_newton=1e-13)
    return cd, ns


def _w8_state(DOF):
    """A smooth coupled state [T | u | v | p] and direction on W8's meshes (the same nodes for CD and NS)."""
    from oracle import sem_oracle as O
    c = W8
    x, y = O.global_nodes(c["P"], c["nex"], c["ney"], 1.0 / c["nex"], 1.0 / c["ney"])
    s = np.sin(np.pi * x) * np.sin(np.pi * y)
    state = np.concatenate((0.5 - x, 0.05 * s * np.cos(np.pi * y), -0.05 * s * np.cos(np.pi * x), 0.01 * x * y))
    d = np.concatenate((0.1 * s, 0.01 * s * y, -0.01 * s * x, 0.01 * np.cos(np.pi * x) * np.cos(np.pi * y)))
    assert state.size == DOF
    return state, d


def _worker_w8(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch as _torch
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)
    _torch.set_num_threads(1)
    try:
        from cpu_mesh import CPUStripMesh
        from sem_amd.solvers.boussinesq import partitioned_coupler
        c = W8
        cp = partitioned_coupler(dist, 1.0, 1.0, c["Re"], c["Ra"], c["Pr"], c["P"], c["nex"], c["ney"], c["P"], c["nex"],
                                 c["ney"], mesh_factory=CPUStripMesh, mode="JNK")
        x, dx = _w8_state(cp.DOF)
        R = cp.residuals(x)
        cp.linearize(x)
        JR = cp.jacobian_apply(dx)
        Z = cp.block_jacobi(JR)      # both Newton updates element-partitioned (cfg5's path)
        q.put((rank, R, JR, Z))
    finally:
        dist.destroy_process_group()


def test_element_partitioned_coupler_world8():
    """cfg5's world size over the CPU: both solvers strip-partitioned over 8 ranks on a 9-column mesh (uneven
    strips, seven one-column strips), against the same coupler over one process (the sequential coupler with
    the oracle's solver classes): coupled residual and Jacobian apply to 1e-12, and one block-Jacobi
    preconditioner application -- both Newton updates element-partitioned (StripLineSolver, distributed
    Schur GMRES) -- to the accuracy the solvers' 1e-13 sqrt(N) stopping rule implies.  (The whole coupled
    solve over 8 gloo ranks takes minutes on the CPU; world 2 runs it against the golden below.)"""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    c = W8
    cd, ns = _w8_solvers()
    ref = BoussinesqCoupler(1.0, 1.0, c["Re"], c["Ra"], c["Pr"], c["P"], c["nex"], c["ney"], c["P"], c["nex"], c["ney"],
                            mode="JNK", cd=cd, ns=ns)
    x, dx = _w8_state(ref.DOF)
    R0 = ref.residuals(x)
    ref.linearize(x)
    JR0 = ref.jacobian_apply(dx)
    Z0 = ref.block_jacobi(JR0)
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_w8, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, R, JR, Z in out:
        assert np.abs(R - R0).max() <= 1e-12 * np.abs(R0).max(), rank
        assert np.abs(JR - JR0).max() <= 1e-12 * np.abs(JR0).max(), rank
        # T, u, v of the update; the pressure is unique only up to the equal-order discretisation's spurious
        # mode, so it is held to the looser bar
        nv = ref.Ncd + 2 * ref.Nns
        assert np.abs(Z[:nv] - Z0[:nv]).max() <= 1e-7 * np.abs(Z0[:nv]).max(), rank
        assert np.abs(Z[nv:] - Z0[nv:]).max() <= 1e-4 * np.abs(Z0[nv:]).max(), rank


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
