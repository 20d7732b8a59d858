"""The RCCL ("nccl") branches of the element-partitioned path, executed on one GPU.

RCCL refuses two ranks on one GPU, so every partitioned test on the one-GPU box used gloo, and the
device-resident collective branches -- the ones BASELINE configs[4] and the driver's multi-GPU bench take --
ran only when the driver had an 8-GPU node.  Here ONE spawned process initialises a real one-rank RCCL process
group on cuda:0 and drives those branches:

  world 1 (the real group):   Partition collectives on the device (norm, amax, broadcast, gather, the Krylov
                              reduce without host staging), the pipelined partitioned GMRES with the device reduce
                              (against plain GMRES, with and without forced reorthogonalisation), the partitioned
                              CD and NS solvers against the whole-mesh ones, the _StripSchur hipGraph capture with
                              its agreement all-reduces, the strip solve with refinement forced on;
  rank 0 (and 1) of 2 (tests/rank_view.py over the same group): the G >= 2 branches -- bench.py's N > 1 step
                              (position-ranged applies, interface pack, async RCCL all-reduce, unpack) captured
                              exactly as bench.time_steps captures it, with the all-ranks capture-agreement
                              all-reduce; InterfaceExchange.many; the strip velocity solver's G = 2 factor (RCCL
                              all-gather of the reduced blocks), its graph capture, and the G = 2 _StripSchur
                              capture.  A one-rank sum is the local tensor, so the exchange is checked bitwise
                              against the no-exchange apply and the graphs against eager execution.
The branches only G >= 2 REAL ranks reach (values from other ranks, p2p send/recv with a neighbour) stay
covered by the gloo tests and are listed in DESIGN.md section 7 as unverified until the driver's SCALE run.
"""
import json
import os
import socket
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NS_CASE = dict(P=4, nex=6, ney=4, Re=100.0, Gr=50.0)
CD_CASE = dict(P=6, nex=12, ney=7, Pe=40.0)


def _rel(a, b):
    a, b = (t.double().cpu() if isinstance(t, torch.Tensor) else torch.as_tensor(t, dtype=torch.float64)
            for t in (a, b))
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-300))


# --------------------------------------------------------------------------- scenarios (run in the worker)
def sc_bench_step(dist, dev):
    """bench.py's N > 1 step as rank r of 2 strips: graph replay bitwise equal to the eager step, and the
    exchanged result bitwise equal to the strip apply alone (a one-rank all-reduce sums nothing)."""
    import bench
    out = {}
    for rank in (0, 1):
        for overlap in (True, False):
            step, mesh, (T, y, kw), _ = bench.build_strip_step(8, 64, 32, 1.0 / 32, 40.0, 2, rank, dev, dist,
                                                                 overlap=overlap, seed=2024 + rank)
            y.zero_()
            step()
            torch.cuda.synchronize(dev)
            y_eager = y.clone()
            y_plain = mesh.apply(T, **kw)
            y.zero_()
            secs, used = bench.time_steps(step, 30, 3, dev, use_graph=True, dist=dist)
            key = f"r{rank}_{'overlap' if overlap else 'serial'}"
            out[key] = dict(graph=used, graph_eq_eager=bool(torch.equal(y, y_eager)),
                            exchange_identity=bool(torch.equal(y_eager, y_plain)), us_per_step=secs / 30 * 1e6)
    return out


def sc_interface_many(dist, dev):
    from sem_amd.device import get_mesh
    from sem_amd.parallel import StripPartition
    part = StripPartition(16, 2)
    mesh = get_mesh(5, 16, 6, 1.0 / 16, 1.0 / 6, 0, 8, dev.index)
    ys = [torch.rand(mesh.n_local, dtype=torch.float64, device=dev) for _ in range(3)]
    want = [y.clone() for y in ys]
    ex = part.exchanger(mesh, dist, kind="allreduce")
    ex.many(ys)
    ex(ys[0])
    torch.cuda.synchronize(dev)
    return dict(unchanged=all(torch.equal(a, b) for a, b in zip(ys, want)))


def sc_partition_collectives(dist, dev):
    from sem_amd.parallel import Partition
    c = CD_CASE
    part = Partition(dist)
    mesh = part.setup(c["P"], c["nex"], c["ney"], 1.0 / c["nex"], 1.0 / c["ney"])
    a, b = (torch.rand(mesh.n_local, dtype=torch.float64, device=dev) * 2 - 1 for _ in range(2))
    t = torch.rand(5, dtype=torch.float64, device=dev)
    t0 = t.clone()
    n0 = part.inner.collectives
    part.inner.reduce(t)
    h = part.inner(torch.stack((a, b)), a)
    return dict(world=part.world, backend_device=str(part.backend_device()), inner_bdev=str(part.inner.bdev),
                norm=_rel(part.norm(a, b), torch.sqrt(a.square().sum() + b.square().sum())),
                amax=_rel(part.amax(a, b), torch.maximum(a.abs().max(), b.abs().max())),
                gather=bool(torch.equal(part.gather(a), a)),
                broadcast=bool(torch.equal(part.broadcast(b.cpu()), b.cpu())),
                reduce_identity=bool(torch.equal(t, t0)), reduce_count=part.inner.collectives - n0,
                inner=_rel(h, torch.stack((a, b)) @ a))


def sc_pipelined_gmres(dist, dev):
    """Partitioned GMRES with the device-resident RCCL reduce (pipelined: no host staging) against plain GMRES."""
    from sem_amd import _lib, krylov
    from sem_amd.parallel import Partition
    c = CD_CASE
    part = Partition(dist)
    mesh = part.setup(c["P"], c["nex"], c["ney"], 1.0 / c["nex"], 1.0 / c["ney"])
    r = np.random.default_rng(11)
    u, v, b = (mesh.to_device(r.uniform(-1, 1, mesh.n_local)) for _ in range(3))
    kw = dict(c_stiff=1.0, c_gradx=c["Pe"], cu=u, c_grady=c["Pe"], cv=v, dir_mode=_lib.DIR_IDENTITY,
              dir_sides=_lib.SIDE_W | _lib.SIDE_E)
    out = {}
    for eta in (None, 2.0):   # 2.0: an extra orthogonalisation pass at every step (the reorthogonalisation branch)
        old = krylov.REORTH_ETA
        if eta is not None:
            krylov.REORTH_ETA = eta
        try:
            ref = krylov.gmres(lambda x: mesh.apply(x, **kw), b, atol=1e-11, restart=60, maxiter=20000)
            n0 = part.inner.collectives
            got = krylov.gmres(lambda x: mesh.apply(x, **kw), b, atol=1e-11, restart=60, maxiter=20000,
                               inner=part.inner)
        finally:
            krylov.REORTH_ETA = old
        out["reorth" if eta else "plain"] = dict(
            info=got.info, iters=got.iters, ref_iters=ref.iters, x=_rel(got.x, ref.x), reorth=got.reorth,
            discarded=got.discarded, collectives=part.inner.collectives - n0)
    return out


def sc_cd_solver(dist, dev):
    from sem_amd.parallel import Partition
    from sem_amd.solvers import ConvectionDiffusionSolver
    c = CD_CASE
    args = (1.0, 1.0, c["Pe"], c["P"], c["nex"], c["ney"])
    whole = ConvectionDiffusionSolver(*args, T_W=0.5, T_E=-0.5, mtol=1e-10)
    part = ConvectionDiffusionSolver(*args, T_W=0.5, T_E=-0.5, mtol=1e-10, partition=Partition(dist))
    r = np.random.default_rng(23)
    T, u, v, dT, du, dv = (r.uniform(-1, 1, whole.N) for _ in range(6))
    out = {}
    for name, s in (("whole", whole), ("part", part)):
        res = s._get_residuals(T, u, v)
        s._calc_jacobians(T)
        dres = s._get_dresiduals(dT, du, dv)
        sol = s._get_solution(s.points[1] - 0.5, 0.5 - s.points[0])
        out[name] = (res, dres, sol)
    return dict(res=_rel(out["part"][0], out["whole"][0]), dres=_rel(out["part"][1], out["whole"][1]),
                sol=float(np.abs(out["part"][2] - out["whole"][2]).max()))


def _ns_fields(N):
    r = np.random.default_rng(41)
    return [r.uniform(-1, 1, N) for _ in range(7)]


def sc_ns_solver(dist, dev):
    """NavierStokesSolver(partition=Partition(one-rank RCCL group)): the distributed update (strip velocity solver,
    _StripSchur captured with its agreement all-reduces, partitioned GMRES on the device reduce) against the whole-
    mesh solver; then the strip solve with refinement forced on."""
    from sem_amd.parallel import Partition
    from sem_amd.solvers import NavierStokesSolver
    from sem_amd.solvers.navier_stokes import _StripSchur
    c = NS_CASE
    args = (1.0, 1.0, c["Re"], c["Gr"], c["P"], c["nex"], c["ney"])
    kw = dict(u_N=1.0, mtol=1e-10, mtol_newton=1e-9, iprint=[])
    res = {}
    for name, part in (("whole", None), ("part", Partition(dist))):
        ns = NavierStokesSolver(*args, partition=part, **kw)
        u, v, p, T, du, dv, dp = _ns_fields(ns.N)
        r = {"res": ns._get_residuals(u, v, p, T)}
        ns._calc_jacobians(u, v)
        r["dres"] = ns._get_dresiduals(du, dv, dp, T)
        r["upd"] = ns._get_update(*r["res"])
        r["sol"] = ns._get_solution(np.zeros(ns.N))
        r["newton"] = ns._k
        res[name] = r
        if part is not None:
            sch = ns._schur
            out = dict(schur_graph=isinstance(sch, _StripSchur) and sch._graph is not None)
            if out["schur_graph"]:
                x = torch.rand(ns._mesh.n_local, dtype=torch.float64, device=dev)
                out["schur_graph_vs_eager"] = _rel(sch(x), ns._schur_strips(ns._velo, x))
            vs = ns._velo
            B = torch.rand((vs.NX, vs.m), dtype=torch.float64, device=dev)
            vs.refine = False
            X0 = vs._solve_lines(B)
            vs.refine = True
            X1 = vs._solve_lines(B)
            J = ns._velocity_apply_lines
            out["refined_resid"] = float((J(X1) - B).abs().max() / B.abs().max())
            out["plain_resid"] = float((J(X0) - B).abs().max() / B.abs().max())
            out["refined_vs_plain"] = _rel(X1, X0)
    w, p = res["whole"], res["part"]
    out["res"] = max(_rel(a, b) for a, b in zip(p["res"], w["res"]))
    out["dres"] = max(_rel(a, b) for a, b in zip(p["dres"], w["dres"]))
    out["upd"] = max(float(np.abs(a - b).max()) for a, b in zip(p["upd"][:2], w["upd"][:2]))
    out["sol"] = max(float(np.abs(a - b).max()) for a, b in zip(p["sol"][:2], w["sol"][:2]))
    out["newton"] = (p["newton"], w["newton"])
    return out


def sc_strip_view(dist, dev):
    """Rank 0 of 2 strips through RankView over the real group: the G = 2 strip velocity factor (RCCL all-gather
    of the reduced blocks), the strip solver's capture (checked against eager inside capture() with agreement
    all-reduces), and the G = 2 _StripSchur capture (gradient assembly by RCCL all-reduce, the all-gather of the
    boundary right-hand sides, divergence assembly -- all inside one hipGraph)."""
    from rank_view import RankView
    from sem_amd.parallel import Partition
    from sem_amd.solvers import NavierStokesSolver
    from sem_amd.solvers.navier_stokes import _StripSchur
    c = NS_CASE
    out = {}
    for r in (0, 1):
        view = RankView(dist, 2, r)
        ns = NavierStokesSolver(1.0, 1.0, c["Re"], c["Gr"], c["P"], c["nex"], c["ney"], u_N=1.0, mtol=1e-10,
                                mtol_newton=1e-9, iprint=[], partition=Partition(view))
        u, v, p, T, _, _, _ = _ns_fields(ns.N)
        ns._get_residuals(u, v, p, T)
        ns._calc_jacobians(u, v)
        vs = ns._strip_velocity_solver()
        vs.refine = False          # the stand-in reduced blocks make the refinement probe meaningless
        g0 = dict(view.calls)
        cap = vs.capture()
        B = torch.rand((vs.NX, vs.m), dtype=torch.float64, device=dev)
        want = vs._solve_lines(B.clone())
        vs._bin.copy_(B)
        if cap:
            vs._graph.replay()
        solve_eq = _rel(vs._xout, want) if cap else None
        vs._graph = None
        sch = _StripSchur(ns, vs, graph=True)
        x = torch.rand(ns._mesh.n_local, dtype=torch.float64, device=dev)
        sch_err = _rel(sch(x), ns._schur_strips(vs, x)) if sch._graph is not None else None
        out[f"r{r}"] = dict(strip=[ns._mesh.ex_begin, ns._mesh.ex_end], solve_graph=cap, solve_graph_vs_eager=solve_eq,
                            schur_graph=sch._graph is not None, schur_graph_vs_eager=sch_err,
                            gathers=view.calls.get("all_gather", 0), gathers_before_capture=g0.get("all_gather", 0),
                            all_reduces=view.calls.get("all_reduce", 0))
    return out


SCENARIOS = {"bench_step": sc_bench_step, "interface_many": sc_interface_many,
             "partition_collectives": sc_partition_collectives, "pipelined_gmres": sc_pipelined_gmres,
             "cd_solver": sc_cd_solver, "ns_solver": sc_ns_solver, "strip_view": sc_strip_view}


def _worker(port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.set_num_threads(8)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    results = {"backend": dist.get_backend()}
    try:
        for name, fn in SCENARIOS.items():
            try:
                results[name] = ("ok", fn(dist, dev))
            except Exception:   # report the failure, keep going: one broken branch must not hide the others
                results[name] = ("error", traceback.format_exc())
            print(f"[rccl worker] {name}: {results[name][0]}", flush=True)
    finally:
        q.put(results)
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0, p.exitcode
    print(json.dumps({k: (v if k == "backend" else {"status": v[0], "result": v[1]}) for k, v in out.items()},
                     default=str), flush=True)     # the record (pytest -s / the log of a -v run on failure)
    return out


def _get(rccl, name):
    status, val = rccl[name]
    assert status == "ok", val
    return val


def test_backend_is_rccl(rccl):
    assert rccl["backend"] == "nccl"


def test_bench_step_capture_over_rccl(rccl):
    for key, r in _get(rccl, "bench_step").items():
        assert r["graph"], key                   # every rank agreed that its capture succeeded
        assert r["graph_eq_eager"], key          # bitwise
        assert r["exchange_identity"], key       # pack -> one-rank RCCL all-reduce -> unpack is the identity


def test_interface_exchange_many_over_rccl(rccl):
    assert _get(rccl, "interface_many")["unchanged"]


def test_partition_device_collectives(rccl):
    r = _get(rccl, "partition_collectives")
    assert r["world"] == 1 and r["backend_device"].startswith("cuda") and r["inner_bdev"] == "cuda"
    assert r["norm"] < 1e-14 and r["amax"] == 0.0 and r["inner"] < 1e-14
    assert r["gather"] and r["broadcast"] and r["reduce_identity"] and r["reduce_count"] == 2   # reduce + inner


def test_pipelined_gmres_device_reduce(rccl):
    for key, r in _get(rccl, "pipelined_gmres").items():
        assert r["info"] == 0, key
        assert abs(r["iters"] - r["ref_iters"]) <= 1, (key, r)
        assert r["x"] < 1e-9, (key, r)
        assert r["discarded"] >= 1, (key, r)     # the pipelined step ran (its speculation past convergence dropped)
        assert r["collectives"] >= 2 * r["iters"], (key, r)
    assert _get(rccl, "pipelined_gmres")["reorth"]["reorth"] >= 1


def test_partitioned_cd_solver_over_rccl(rccl):
    r = _get(rccl, "cd_solver")
    assert r["res"] <= 1e-13 and r["dres"] <= 1e-13, r
    assert r["sol"] < 1e-8, r


def test_partitioned_ns_solver_over_rccl(rccl):
    r = _get(rccl, "ns_solver")
    assert r["res"] <= 1e-13 and r["dres"] <= 1e-13, r
    assert r["schur_graph"], r
    assert r["schur_graph_vs_eager"] <= 1e-12, r
    # two Schur Krylov solves (all-reduced against plain inner products) stopped at the reference's absolute tolerance
    # mtol sqrt(N) = 2e-9 agree to that tolerance times the Schur system's conditioning (1.1e-8 measured with the
    # nested-dissection velocity solves); the converged Newton solutions agree tighter
    assert r["upd"] < 5e-8 and r["sol"] < 1e-8, r
    assert r["newton"][0] == r["newton"][1], r
    assert r["refined_resid"] <= max(2 * r["plain_resid"], 1e-13), r
    assert r["refined_vs_plain"] < 1e-8, r


def test_strip_solver_g2_capture_over_rccl(rccl):
    for key, r in _get(rccl, "strip_view").items():
        assert r["gathers_before_capture"] >= 1, (key, r)     # the reduced blocks went through the RCCL all-gather
        assert r["solve_graph"], (key, r)
        assert r["solve_graph_vs_eager"] <= 1e-12, (key, r)
        assert r["schur_graph"], (key, r)
        assert r["schur_graph_vs_eager"] <= 1e-12, (key, r)
