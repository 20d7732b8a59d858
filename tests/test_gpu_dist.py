"""Strip-partitioned solve on the device: two ranks on one GPU (gloo for the collectives, the
only backend that runs several ranks on one device), real band-kernel applies, real
interface pack/unpack kernels, DistributedInner dot products -- against the single-domain
device solve.  The RCCL path differs only in the backend string (bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
P, NEX, NEY, PE = 6, 12, 7, 40.0


def _inputs():
    N = (NEX * P + 1) * (NEY * P + 1)
    r = np.random.default_rng(11)
    return r.uniform(-1, 1, N), r.uniform(-1, 1, N), r.uniform(-1, 1, N)


def _solve(mesh, u, v, b, exch=None, inner=None):
    from sem_amd import _lib
    from sem_amd.krylov import gmres
    U, V, B = (mesh.to_device(a) for a in (u, v, b))
    kw = dict(c_stiff=1.0, c_gradx=PE, cu=U, c_grady=PE, cv=V, dir_mode=_lib.DIR_IDENTITY,
              dir_sides=_lib.SIDE_W | _lib.SIDE_E)

    def mv(x):
        y = mesh.apply(x, **kw)
        return exch(y) if exch is not None else y

    return gmres(mv, B, atol=1e-11, restart=60, maxiter=20000, inner=inner)


def _worker(rank, world, port, q, kind):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 16 // world))   # ranks share the box's CPU share: no OpenMP oversubscription
    try:
        from sem_amd.device import get_mesh
        from sem_amd.parallel import DistributedInner, StripPartition
        part = StripPartition(NEX, world)
        eb, ee = part.local_range(rank)
        mesh = get_mesh(P, NEX, NEY, 1.0 / NEX, 1.0 / NEY, eb, ee, 0)
        u, v, b = _inputs()
        sl = slice(mesh.dof_begin, mesh.dof_begin + mesh.n_local)
        res = _solve(mesh, u[sl], v[sl], b[sl], exch=part.exchanger(mesh, dist, kind=kind),
                     inner=DistributedInner(part, mesh, dist))
        q.put((rank, res.info, res.iters, mesh.dof_begin, res.x.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_device_gmres(gpu, world):
    from sem_amd.device import get_mesh
    u, v, b = _inputs()
    ref = _solve(get_mesh(P, NEX, NEY, 1.0 / NEX, 1.0 / NEY), u, v, b)
    assert ref.info == 0
    xr = ref.x.cpu().numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "allreduce")) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, info, iters, d0, x in out:
        assert info == 0 and abs(iters - ref.iters) <= max(2, ref.iters // 50), (rank, iters, ref.iters)
        assert np.abs(x - xr[d0:d0 + len(x)]).max() < 1e-8 * max(1.0, np.abs(xr).max())


def _worker_solver(rank, world, port, q, kind, overlap):
    """ConvectionDiffusionSolver(partition=...) on real strip meshes: residual / Jacobian applies
    and the Newton step with the partitioned device GMRES."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 16 // world))   # ranks share the box's CPU share: no OpenMP oversubscription
    try:
        from sem_amd.parallel import Partition
        from sem_amd.solvers import ConvectionDiffusionSolver
        part = Partition(dist, exchange=kind, overlap=overlap)
        cd = ConvectionDiffusionSolver(1.0, 1.0, PE, P, NEX, NEY, T_W=0.5, T_E=-0.5, mtol=1e-10, partition=part)
        r = np.random.default_rng(23)
        T, u, v, dT, du, dv = (r.uniform(-1, 1, cd.N) for _ in range(6))
        res = cd._get_residuals(T, u, v)
        cd._calc_jacobians(T)
        dres = cd._get_dresiduals(dT, du, dv)
        pts = cd.points
        sol = cd._get_solution(pts[1] - 0.5, 0.5 - pts[0])
        q.put((rank, res, dres, sol, cd.matvecs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,overlap", [(2, "allreduce", True), (3, "allreduce", True), (3, "p2p", True),
                                                (2, "allreduce", False)])
def test_partitioned_cd_solver(gpu, world, kind, overlap):
    from sem_amd.solvers import ConvectionDiffusionSolver
    # the whole-mesh solver with its condensed direct preconditioner; the partitioned solver's GMRES is
    # preconditioned by the element-partitioned condensation of the same Jacobian (strip_solve.py), so
    # both take one or two matvecs
    cd = ConvectionDiffusionSolver(1.0, 1.0, PE, P, NEX, NEY, T_W=0.5, T_E=-0.5, mtol=1e-10)
    r = np.random.default_rng(23)
    T, u, v, dT, du, dv = (r.uniform(-1, 1, cd.N) for _ in range(6))
    res = cd._get_residuals(T, u, v)
    cd._calc_jacobians(T)
    dres = cd._get_dresiduals(dT, du, dv)
    pts = cd.points
    sol = cd._get_solution(pts[1] - 0.5, 0.5 - pts[0])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_solver, args=(rr, world, port, q, kind, overlap)) for rr in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, pres, pdres, psol, mv in out:
        assert np.abs(pres - res).max() <= 1e-13 * np.abs(res).max(), rank
        assert np.abs(pdres - dres).max() <= 1e-13 * np.abs(dres).max(), rank
        assert np.abs(psol - sol).max() < 1e-8, rank
        assert mv <= cd.matvecs + 2 <= 5, (rank, mv, cd.matvecs)


NS_CASE = dict(P=4, nex=6, ney=4, Re=100.0, Gr=50.0)


def _ns_fields(N):
    r = np.random.default_rng(41)
    return [r.uniform(-1, 1, N) for _ in range(7)]


def _ns_run(ns):
    """The NS solver methods the Boussinesq coupler calls, at a seeded state, then a lid-driven solve."""
    u, v, p, T, du, dv, dp = _ns_fields(ns.N)
    out = {"res": ns._get_residuals(u, v, p, T)}
    ns._calc_jacobians(u, v)
    out["dres"] = ns._get_dresiduals(du, dv, dp, T)
    z = np.zeros(ns.N)
    out["sol"] = ns._get_solution(z)
    out["newton"] = ns._k
    return out


def _worker_ns(rank, world, port, q, kind):
    """NavierStokesSolver(partition=...) on real strip meshes (the fused strip sem_ns_apply, interface
    assembly of the three outputs in one collective); Newton updates by the element-partitioned velocity
    condensation (sem_condensed_blocks on strip handles, StripLineSolver) inside the strip Schur GMRES."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 16 // world))   # ranks share the box's CPU share: no OpenMP oversubscription
    try:
        from sem_amd.parallel import Partition
        from sem_amd.solvers import NavierStokesSolver
        c = NS_CASE
        ns = NavierStokesSolver(1.0, 1.0, c["Re"], c["Gr"], c["P"], c["nex"], c["ney"], u_N=1.0, mtol=1e-10,
                                mtol_newton=1e-9, iprint=[], partition=Partition(dist, exchange=kind))
        q.put((rank, _ns_run(ns)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "allreduce"), (3, "p2p")])
def test_partitioned_ns_solver(gpu, world, kind):
    from sem_amd.solvers import NavierStokesSolver
    c = NS_CASE
    ns = NavierStokesSolver(1.0, 1.0, c["Re"], c["Gr"], c["P"], c["nex"], c["ney"], u_N=1.0, mtol=1e-10,
                            mtol_newton=1e-9, iprint=[])
    want = _ns_run(ns)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_ns, args=(r, world, port, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got in out:
        for key in ("res", "dres"):
            for a, b in zip(got[key], want[key]):
                assert np.abs(a - b).max() <= 1e-13 * np.abs(b).max(), (rank, key)
        assert got["newton"] == want["newton"], rank
        for a, b in zip(got["sol"][:2], want["sol"][:2]):
            assert np.abs(a - b).max() < 1e-8, rank


CFG5 = dict(P=12, ne=128, Re=1e3, Ra=1e6, Pr=0.71)


def _cfg5_state(DOF):
    r = np.random.default_rng(55)
    return r.uniform(-0.5, 0.5, DOF), r.uniform(-1, 1, DOF)


def _worker_cfg5(rank, world, port, q):
    """BASELINE cfg5's element-partitioned coupler (128^2, P=12, both solvers strip-partitioned): one
    coupled residual and Jacobian apply (every apply a strip launch + interface exchange)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 16 // world))   # ranks share the box's CPU share: no OpenMP oversubscription
    try:
        from sem_amd.solvers.boussinesq import partitioned_coupler
        c5 = CFG5
        c = partitioned_coupler(dist, 1.0, 1.0, c5["Re"], c5["Ra"], c5["Pr"], c5["P"], c5["ne"], c5["ne"], c5["P"],
                                c5["ne"], c5["ne"])
        x, dx = _cfg5_state(c.DOF)
        R = c.residuals(x)
        c.linearize(x)
        JR = c.jacobian_apply(dx)
        if rank == 0:
            q.put((R, JR))
    finally:
        dist.destroy_process_group()


def test_cfg5_element_partitioned_coupled_maps(gpu):
    """cfg5 (128^2, P=12, 9.45 M coupled DOFs) split over 4 ranks on one GPU: the partitioned coupled
    residual and Jacobian apply equal the whole-mesh device coupler's to 1e-13 (the whole-mesh maps are
    pinned to the reference at small sizes and by cfg5_checksums.npz at this size)."""
    from sem_amd.solvers.boussinesq import BoussinesqCoupler
    c5 = CFG5
    c = BoussinesqCoupler(1.0, 1.0, c5["Re"], c5["Ra"], c5["Pr"], c5["P"], c5["ne"], c5["ne"], c5["P"], c5["ne"],
                          c5["ne"])
    x, dx = _cfg5_state(c.DOF)
    R = c.residuals(x)
    c.linearize(x)
    JR = c.jacobian_apply(dx)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_worker_cfg5, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    PR, PJR = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.abs(PR - R).max() <= 1e-13 * np.abs(R).max()
    assert np.abs(PJR - JR).max() <= 1e-13 * np.abs(JR).max()


def _worker_strip_velocity(rank, world, port, q, case):
    """StripLineSolver on real strip handles: sem_condensed_blocks writes the strip's partial pieces, each
    rank condenses its own columns, the reduced system over the strip-boundary lines is shared."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 16 // world))   # ranks share the box's CPU share: no OpenMP oversubscription
    try:
        from velocity_blocks import oracle_velocity_jacobian
        import scipy.sparse.linalg as spla
        from sem_amd import _lib
        from sem_amd.device import get_mesh
        from sem_amd.parallel import StripPartition
        from sem_amd.solvers.strip_solve import StripLineSolver
        P, nex, ney, Re = case
        ref, u, v = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
        part = StripPartition(nex, world)
        eb, ee = part.local_range(rank)
        mesh = get_mesh(P, nex, ney, 1.0 / nex, 1.0 / ney, eb, ee, 0)
        sl = slice(mesh.dof_begin, mesh.dof_begin + mesh.n_local)
        d = lambda a: mesh.to_device(np.asarray(a)[sl])  # noqa: E731
        kw = dict(c_stiff=1.0, c_gradx=Re, cu=d(u), c_grady=Re, cv=d(v), juu=d(Re * (ref.Gx @ u)),
                  jvv=d(Re * (ref.Gy @ v)), juv=d(Re * (ref.Gy @ u)), jvu=d(Re * (ref.Gx @ v)),
                  dir_sides=_lib.SIDE_W | _lib.SIDE_E | _lib.SIDE_S | _lib.SIDE_N)
        vs = StripLineSolver(P, nex, ney, mesh.device, part.bounds, rank, dist, gather_device="cpu")
        vs.factor_mesh(mesh, budget_bytes=1, **kw)     # one column per chunk
        r = np.random.default_rng(3)
        bu, bv = r.uniform(-1, 1, ref.N), r.uniform(-1, 1, ref.N)
        want = spla.spsolve(ref.Jvelo.tocsc(), np.hstack((bu, bv)))
        xu, xv = vs.solve(d(bu), d(bv))
        err = max(np.abs(xu.cpu().numpy() - want[:ref.N][sl]).max(), np.abs(xv.cpu().numpy() - want[ref.N:][sl]).max())
        q.put((rank, err / np.abs(want).max(), sl.start, xu.cpu().numpy(), xv.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, (4, 4, 3, 300.0)), (3, (6, 7, 2, 1000.0)), (2, (12, 2, 3, 500.0))])
def test_strip_velocity_solve_real_kernels(gpu, world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_strip_velocity, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, *_ in out:
        assert err <= 1e-9, (rank, err)
    # backward error of the assembled strip solution with the reference's own Jacobian: the
    # forward error above is bounded by cond(J) times this
    from velocity_blocks import oracle_velocity_jacobian
    P, nex, ney, Re = case
    ref, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
    xu, xv = np.zeros(ref.N), np.zeros(ref.N)
    for _, _, start, lu, lv in out:      # shared lines hold equal values on both ranks
        xu[start:start + lu.size], xv[start:start + lv.size] = lu, lv
    r = np.random.default_rng(3)
    b = np.hstack((r.uniform(-1, 1, ref.N), r.uniform(-1, 1, ref.N)))
    J, x = ref.Jvelo.tocsr(), np.hstack((xu, xv))
    eta = np.abs(J @ x - b).max() / (abs(J).sum(axis=1).max() * np.abs(x).max() + np.abs(b).max())
    print(f"strip solve over {world} ranks: backward error {eta:.1e}")
    assert eta <= 1e-13, eta


MTOL5 = 1e-13   # the couplers' mtol_internal (Boussinesq_SequentialCoupler.py:61-63)


def _smooth_step(x, y):
    """A smooth (du, dv, dp) with zero Dirichlet velocities on the walls of the unit square."""
    s = np.sin(np.pi * x) * np.sin(np.pi * y)
    return 1e-2 * s * np.cos(np.pi * y), -1e-2 * s * np.cos(np.pi * x), 1e-2 * np.cos(np.pi * x) * np.cos(np.pi * y)


def _worker_cfg5_update(rank, world, port, q):
    """cfg5's NS block solve element-partitioned (128^2, P=12 over `world` ranks): the velocity Jacobian
    factored by the strips' condensations + the reduced boundary-line system, the Schur GMRES over the
    strips; linearised at a smooth flow (T = 1/2 - x, Ra = 1e6), right-hand side the partitioned Jacobian
    applied to a smooth step (a consistent right-hand side, as a Newton step's is).  Rank 0 reports the
    factorisation time, the Schur iterations with elapsed time (every 25), and the solve."""
    import sys
    import time as _t
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 16 // world))   # ranks share the box's CPU share: no OpenMP oversubscription
    try:
        from sem_amd.parallel import Partition
        from sem_amd.solvers import NavierStokesSolver
        c5 = CFG5
        ns = NavierStokesSolver(1.0, 1.0, c5["Re"], c5["Ra"] / c5["Pr"], c5["P"], c5["ne"], c5["ne"], mtol=MTOL5,
                                mtol_newton=MTOL5, iprint=[], partition=Partition(dist))
        x, y = ns.points                  # this rank's nodes (a partitioned solver's points are its strip's)
        say = (lambda msg: print(f"[cfg5 update rank 0 {_t.strftime('%H:%M:%S')}] {msg}", flush=True)) \
            if rank == 0 else (lambda msg: None)
        say(f"solver built, strip {ns._mesh.ex_begin}..{ns._mesh.ex_end} of {c5['ne']} columns")
        u0, v0, _ = _smooth_step(x, y)
        ns._get_residuals(10 * u0, 10 * v0, np.zeros(ns.N), 0.5 - x)
        ns._calc_jacobians(10 * u0, 10 * v0)
        t0 = _t.perf_counter()
        vs = ns._strip_velocity_solver()
        torch.cuda.synchronize()
        say(f"strip velocity factor {_t.perf_counter() - t0:.1f} s "
            f"({torch.cuda.memory_allocated() / 1e9:.1f} GB on this rank)")
        step = _smooth_step(x, y)
        rhs = [ns._dev(a) for a in ns._get_dresiduals(*step)]
        ns._progress = 25 if rank == 0 else 0
        t0 = _t.perf_counter()
        du, dv, dp = ns._get_update(*rhs)
        torch.cuda.synchronize()
        secs = _t.perf_counter() - t0
        say(f"update {secs:.1f} s, {ns.schur_matvecs} Schur matvecs ({1e3 * secs / max(1, ns.schur_matvecs):.1f} ms "
            f"per matvec incl. GMRES)")
        lin = ns._get_dresiduals(du, dv, dp)
        err = ns._norm(*(a - b for a, b in zip(lin, rhs)))
        # velocity error relative to the step's largest velocity, over all ranks (max-reduced)
        e = torch.tensor([float((du - ns._dev(step[0])).abs().max()), float((dv - ns._dev(step[1])).abs().max()),
                          float(max(np.abs(step[0]).max(), np.abs(step[1]).max()))], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        verr = float(max(e[0], e[1]) / e[2])
        say(f"residual {err:.3e} (tolerance {MTOL5:g} sqrt(N) = {MTOL5 * np.sqrt(ns.N):.3e}), "
            f"velocity error against the step {verr:.2e} (relative)")
        if rank == 0:
            q.put((err, MTOL5 * np.sqrt(ns.N), ns.schur_matvecs, secs, verr))
    finally:
        dist.destroy_process_group()


def test_cfg5_element_partitioned_ns_update(gpu):
    """One cfg5 NS Newton update (_get_update) element-partitioned over 4 ranks on one GPU: it solves the
    partitioned Jacobian (the coupled maps above pin that to the whole-mesh device maps) to the reference's
    Schur tolerance mtol sqrt(N) (NavierStokes_Solver.py:222-224)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_worker_cfg5_update, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    err, tol, nmv, secs, verr = q.get(timeout=660)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    print(f"cfg5 partitioned NS update: {nmv} Schur matvecs, {secs:.1f} s, residual {err:.3e} (tol {tol:.3e}), "
          f"velocity error {verr:.2e}")
    # the reference's stopping rule itself, mtol sqrt(N) (NavierStokes_Solver.py:222-224), on the linearised residual
    # of all three equations, and the step's velocities to the accuracy that rule implies (the cfg4 test's bar)
    assert err <= tol and verr < 2e-5
