"""Where the element-partitioned NS Schur matvec spends its time.

Two modes, both on one MI355X:

  rehearsal  -- under torch.distributed.run with W gloo ranks sharing the GPU (the only multi-rank run a
               one-GPU box allows): the partitioned NS solver at one linearisation, K eager Schur matvecs and
               a fixed number of partitioned GMRES iterations, split into the phases of sem_amd.tracing
               (HIP events: device time; host wall with a synchronisation at each phase end), with every
               torch.distributed call counted and its host wall timed.  Run once with the Krylov on the HIP
               sweeps (default) and once on the torch route (--krylov generic) for the before/after.
  solo       -- ONE process as rank r of G (a loopback process group: collectives become local no-ops or
               copies with the real shapes, so the rank does exactly its own device work, uncontended): the
               strip factor time, the eager phase split of one matvec, the graph-captured matvec (the RCCL
               path's shape minus the collectives' latency), the Krylov step's sweeps over the strip, and the
               collectives per matvec / per Krylov step that an 8-GPU run adds.  Optionally the whole-mesh
               matvec in the same process for comparison.

Writes one JSON record per rank (rehearsal) or per simulated rank (solo) to --out (JSON lines).
The reference runs all of this in one process (NavierStokes_Solver.py:176-236, SuperLU + LGMRES).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def smooth_step(x, y):
    s = np.sin(np.pi * x) * np.sin(np.pi * y)
    return 1e-2 * s * np.cos(np.pi * y), -1e-2 * s * np.cos(np.pi * x), 1e-2 * np.cos(np.pi * x) * np.cos(np.pi * y)


class _Work:
    def wait(self):
        return True


class LoopbackDist:
    """A process group of G ranks of which only rank r exists: all_reduce / broadcast / barrier do nothing,
    all_gather copies the local tensor into every slot.  The shapes, and so the device work of rank r, are the
    real ones; the values from "other ranks" are not (timing only).  Backend "nccl": the device-resident
    collective path (no host staging) and the graph captures, as under RCCL."""

    ReduceOp = torch.distributed.ReduceOp

    def __init__(self, G, r):
        self.G, self.r = G, r
        self.calls = {}

    def _count(self, k, t=None):
        c = self.calls.setdefault(k, [0, 0])
        c[0] += 1
        c[1] += 0 if t is None else t.numel() * t.element_size()

    def get_world_size(self, group=None):
        return self.G

    def get_rank(self, group=None):
        return self.r

    def get_backend(self, group=None):
        return "nccl"

    def get_global_rank(self, group, r):
        return r

    def all_reduce(self, t, op=None, group=None, async_op=False):
        self._count("all_reduce", t)
        return _Work() if async_op else None

    def all_gather(self, out, t, group=None, async_op=False):
        self._count("all_gather", t)
        for o in out:
            o.copy_(t)
        return _Work() if async_op else None

    def broadcast(self, t, src=0, group=None, async_op=False):
        self._count("broadcast", t)
        return _Work() if async_op else None

    def barrier(self, group=None):
        self._count("barrier")


def count_collectives(dist):
    """Wrap torch.distributed's collectives: calls, bytes and host wall per kind (rehearsal mode)."""
    stats = {}
    for name in ("all_reduce", "all_gather", "broadcast", "barrier", "batch_isend_irecv"):
        fn = getattr(dist, name)

        def wrap(*a, _fn=fn, _name=name, **kw):
            t0 = time.perf_counter()
            r = _fn(*a, **kw)
            s = stats.setdefault(_name, [0, 0, 0.0])
            s[0] += 1
            t = a[0] if a and isinstance(a[0], torch.Tensor) else (a[1] if len(a) > 1 and isinstance(a[1], torch.Tensor)
                                                                     else None)
            s[1] += 0 if t is None else t.numel() * t.element_size()
            s[2] += time.perf_counter() - t0
            return r
        setattr(dist, name, wrap)
    return stats


def build_solver(dist, ne, P, backend_dev=None, interior="auto"):
    from sem_amd.parallel import Partition
    from sem_amd.solvers import NavierStokesSolver
    ns = NavierStokesSolver(1.0, 1.0, 1e3, 1e6 / 0.71, P, ne, ne, mtol=1e-13, mtol_newton=1e-13, iprint=[],
                            partition=Partition(dist) if dist is not None else None, velocity_interior=interior)
    x, y = ns.points
    u0, v0, _ = smooth_step(x, y)
    ns._get_residuals(10 * u0, 10 * v0, np.zeros(ns.N), 0.5 - x)
    ns._calc_jacobians(10 * u0, 10 * v0)
    return ns, (x, y)


def phase_table(trace, per):
    return {k: {"calls": c, "device_ms": d, "host_ms": h} for k, c, d, h in trace.table(per)}


def time_eager_matvecs(ns, vs, reps, dev):
    from sem_amd import tracing
    dp = torch.rand(ns._mesh.n_local, dtype=torch.float64, device=dev)
    ns._schur_strips(vs, dp)                    # warm-up
    torch.cuda.synchronize(dev)
    tr = tracing.Trace(dev, sync=True)
    t0 = time.perf_counter()
    with tracing.tracing(tr):
        for _ in range(reps):
            with tracing.phase("schur.matvec"):
                ns._schur_strips(vs, dp)
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / reps
    return wall, phase_table(tr, reps)


def krylov_run(ns, vs, iters, dev, generic, trace_on=True):
    """`iters` iterations of the partitioned Schur GMRES (no convergence expected: maxiter = iters), traced."""
    from sem_amd import tracing
    from sem_amd.krylov import gmres
    from sem_amd.solvers.navier_stokes import _StripSchur
    part = ns._part
    schur = _StripSchur(ns, vs, graph=ns._velocity_graph)
    g = torch.Generator(device=dev).manual_seed(3)
    b = torch.rand(ns._mesh.n_local, dtype=torch.float64, device=dev, generator=g)
    part.assemble(b)
    inner = part.inner if not generic else (lambda A, w: part.inner(A, w))

    def precon(c):
        return c / ns._Mdiag

    tr = tracing.Trace(dev, sync=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    with tracing.tracing(tr) if trace_on else _null():
        r = gmres(schur, b, atol=0.0, rtol=0.0, restart=iters + 1, maxiter=iters, precond=precon, inner=inner)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    return wall, r, (phase_table(tr, max(1, r.iters)) if trace_on else {}), schur._graph is not None


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def rehearsal(args):
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.set_num_threads(max(1, args.threads // world))   # the ranks share the box's CPU share
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    stats = count_collectives(dist)
    say = (lambda m: print(f"[strip_profile r0 {time.strftime('%H:%M:%S')}] {m}", flush=True)) if rank == 0 \
        else (lambda m: None)
    rec = {"mode": "rehearsal", "backend": "gloo", "world": world, "rank": rank, "ne": args.ne, "P": args.P}
    ns, _ = build_solver(dist, args.ne, args.P, interior=args.interior)
    rec["strip"] = [ns._mesh.ex_begin, ns._mesh.ex_end]
    rec["n_local"] = ns._mesh.n_local
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    vs = ns._strip_velocity_solver()
    torch.cuda.synchronize(dev)
    rec["factor_s"] = time.perf_counter() - t0
    rec["refine"], rec["refine_eta"] = bool(vs.refine), vs.refine_eta
    rec["factor_phases"] = dict(getattr(vs, "timing", {}))
    say(f"factor {rec['factor_s']:.2f} s, backward error {vs.refine_eta:.1e}, refine {vs.refine}, "
        f"phases {rec['factor_phases']}")
    if args.refactor:   # a second factorisation of the same linearisation: first-call costs against steady state
        ns._velo = None
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        vs = ns._strip_velocity_solver()
        torch.cuda.synchronize(dev)
        rec["refactor_s"] = time.perf_counter() - t0
        rec["refactor_phases"] = dict(getattr(vs, "timing", {}))
        say(f"refactor {rec['refactor_s']:.2f} s, phases {rec['refactor_phases']}")
    for k in list(stats):
        stats[k][:] = [0, 0, 0.0]
    wall, tab = time_eager_matvecs(ns, vs, args.reps, dev)
    rec["matvec_wall_ms"] = 1e3 * wall
    rec["matvec_phases"] = tab
    rec["matvec_collectives"] = {k: {"calls": v[0] / args.reps, "bytes": v[1] / args.reps,
                                     "host_ms": 1e3 * v[2] / args.reps} for k, v in stats.items() if v[0]}
    say(f"eager matvec {1e3 * wall:.1f} ms")
    for form in (["sweeps", "generic"] if args.krylov == "both" else [args.krylov]):
        for k in list(stats):
            stats[k][:] = [0, 0, 0.0]
        kw, r, ktab, graphed = krylov_run(ns, vs, args.iters, dev, generic=(form == "generic"))
        it = max(1, r.iters)
        rec[f"krylov_{form}"] = {"iters": r.iters, "wall_ms_per_iter": 1e3 * kw / it, "phases": ktab,
                                 "matvec_graph": graphed,
                                 "collectives": {k: {"calls": v[0] / it, "bytes": v[1] / it, "host_ms": 1e3 * v[2] / it}
                                                 for k, v in stats.items() if v[0]}}
        say(f"krylov ({form}) {1e3 * kw / it:.1f} ms per iteration")
    out = [None] * world
    dist.all_gather_object(out, rec)
    if rank == 0 and args.out:
        with open(args.out, "a") as f:
            for o in out:
                f.write(json.dumps(o) + "\n")
    dist.destroy_process_group()


def graph_ms(fn, dev, reps):
    fn()
    torch.cuda.synchronize(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    g.replay()
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize(dev)
        ts.append(a.elapsed_time(b))
    del g
    return float(np.median(ts))


def graph_parts(vs, dev, reps):
    """Device time of the strip solve's pieces, each captured and replayed alone."""
    from sem_amd.solvers.velocity_solve import _gemv
    m, n = vs.m, vs.nex
    B = torch.rand((vs.NX, m), dtype=torch.float64, device=dev)
    g = torch.rand((n + 1, m), dtype=torch.float64, device=dev)
    out = {"solve_lines": graph_ms(lambda: vs._solve_lines(B), dev, reps)}
    if getattr(vs, "interior", "") == "nd":      # nested-dissection strip: its operator bytes per solve
        out["strip_nd_GB"] = vs.bytes_per_solve() / 1e9
    else:
        out["iface_solve"] = graph_ms(lambda: vs._iface_solve(g.clone()), dev, reps)
    if getattr(vs, "_T", None) is not None:
        out["interior_sweep"] = graph_ms(lambda: vs._thomas(g[1:n]), dev, reps)
        X01 = vs._T[1]
        xb2 = torch.rand(2 * m, dtype=torch.float64, device=dev)
        yk = torch.rand((n - 1) * m, dtype=torch.float64, device=dev)
        out["back_substitution_gemv"] = graph_ms(lambda: _gemv(X01.view(-1, X01.shape[-1]), xb2, yk, alpha=-1.0,
                                                               beta=1.0), dev, reps)
        out["back_substitution_GB"] = X01.numel() * 8 / 1e9
    if getattr(vs, "_Z", None) is not None:
        h = torch.rand(vs._Z.shape[1], dtype=torch.float64, device=dev)
        x2 = torch.empty(2 * m, dtype=torch.float64, device=dev)
        out["reduced_rows_gemv"] = graph_ms(lambda: _gemv(vs._Z, h, x2), dev, reps)
        out["reduced_rows_GB"] = vs._Z.numel() * 8 / 1e9
    return out


def loopback_gather(fake):
    """StripLineSolver._all_gather for the loopback group: slot r is this rank's tensor; the other slots copy it,
    and the reduced-system blocks R of the other strips (4-D) get a boosted diagonal -- replicated R blocks would
    leave the last reduced line's Dirichlet rows empty (they belong to the right neighbour).  The values are for
    timing only; the shapes and so the work are the real ones."""
    def gather(self, t):
        if self.G == 1:
            return [t]
        fake._count("all_gather", t)
        out = []
        for j in range(self.G):
            u = t.clone()
            if j != self.rank and t.dim() == 4:
                eye = torch.eye(t.shape[-1], dtype=t.dtype, device=t.device) * t.abs().max()
                u[0, 0] += eye
                u[1, 1] += eye
            out.append(u)
        return out
    return gather


def solo(args):
    from sem_amd import tracing
    from sem_amd.krylov import _DeviceSweeps
    from sem_amd.solvers.strip_solve import _StripReduced
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    recs = []
    for r in [int(t) for t in args.ranks.split(",")]:
        fake = LoopbackDist(args.G, r)
        _StripReduced._all_gather = loopback_gather(fake)     # line and nested-dissection strips alike
        rec = {"mode": "solo", "G": args.G, "rank": r, "ne": args.ne, "P": args.P}
        ns, _ = build_solver(fake, args.ne, args.P, interior=args.interior)
        m = ns._mesh
        rec["strip"] = [m.ex_begin, m.ex_end]
        rec["n_local"] = m.n_local
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        vs = ns._strip_velocity_solver()
        torch.cuda.synchronize(dev)
        rec["factor_s"] = time.perf_counter() - t0
        rec["factor_gb_resident"] = torch.cuda.memory_allocated(dev) / 1e9
        # the loopback group's stand-in reduced blocks make the refinement gate's probe meaningless (it measured a
        # large backward error and switched refinement on, doubling every solve): time the plain solve, as a real
        # partition whose gate passes runs it
        rec["refine_eta_loopback"] = vs.refine_eta
        vs.refine = False
        rec["strip_solver"] = type(vs).__name__
        rec["twisted_interior"] = getattr(vs, "_T", None) is not None and vs._T[0][0] == "twisted"
        fake.calls.clear()
        wall, tab = time_eager_matvecs(ns, vs, args.reps, dev)
        rec["eager_matvec_ms"] = 1e3 * wall
        rec["eager_phases"] = tab
        rec["collectives_per_matvec"] = {k: {"calls": v[0] / (args.reps + 1), "bytes": v[1] / (args.reps + 1)}
                                         for k, v in fake.calls.items()}
        # the RCCL path's shape: the matvec captured in one hipGraph (collectives are loopback no-ops here)
        from sem_amd.solvers.navier_stokes import _StripSchur
        sch = _StripSchur(ns, vs, graph=True)
        rec["matvec_graph"] = sch._graph is not None
        if sch._graph is not None:
            dp = torch.rand(m.n_local, dtype=torch.float64, device=dev)
            for _ in range(3):
                sch(dp)
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                sch(dp)
                b.record()
                torch.cuda.synchronize(dev)
                ts.append(a.elapsed_time(b))
            rec["graph_matvec_ms"] = float(np.median(ts))
        # graph-replayed parts of the strip velocity solve (the eager phase split above includes Python launch
        # gaps; these are device time of each piece alone)
        rec["graph_parts_ms"] = graph_parts(vs, dev, args.reps)
        # Krylov step sweeps over the strip at several basis sizes (device time, one rank's share)
        ks = {}
        for k in (100, 300, 600):
            V = torch.rand((k + 1, m.n_local), dtype=torch.float64, device=dev)
            sw = _DeviceSweeps(V, ns._part.inner.segments)
            w = torch.rand(m.n_local, dtype=torch.float64, device=dev)
            c = torch.rand(k, dtype=torch.float64, device=dev)
            for _ in range(3):
                sw.dot2(k, w, V[k - 1])
                sw.update(k, c, w)
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                sw.dot2(k, w, V[k - 1])
                sw.update(k, c, w)
            b.record()
            torch.cuda.synchronize(dev)
            ks[str(k)] = a.elapsed_time(b) / 20
            del V
        rec["krylov_sweeps_ms_at_k"] = ks
        recs.append(rec)
        print(json.dumps({k: rec[k] for k in ("rank", "strip", "factor_s", "eager_matvec_ms", "graph_matvec_ms")
                          if k in rec}), flush=True)
        del ns, vs, sch
        torch.cuda.empty_cache()
    if args.whole:
        rec = {"mode": "whole", "ne": args.ne, "P": args.P}
        ns, _ = build_solver(None, args.ne, args.P, interior=args.interior)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        vs = ns._velocity_solver()
        torch.cuda.synchronize(dev)
        rec["factor_s"] = time.perf_counter() - t0
        from sem_amd.solvers.navier_stokes import _SchurComplement
        sch = _SchurComplement(ns, vs, graph=True)
        dp = torch.rand(ns._mesh.n_local, dtype=torch.float64, device=dev)
        for _ in range(3):
            sch(dp)
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            sch(dp)
            b.record()
            torch.cuda.synchronize(dev)
            ts.append(a.elapsed_time(b))
        rec["graph_matvec_ms"] = float(np.median(ts))
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "a") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["rehearsal", "solo"], default="rehearsal")
    ap.add_argument("--ne", type=int, default=48)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--iters", type=int, default=40, help="partitioned GMRES iterations traced (rehearsal)")
    ap.add_argument("--krylov", choices=["sweeps", "generic", "both"], default="both")
    ap.add_argument("--G", type=int, default=8, help="solo: ranks of the simulated partition")
    ap.add_argument("--ranks", default="0,3", help="solo: which ranks to run (one after the other)")
    ap.add_argument("--whole", type=int, default=1, help="solo: also time the whole-mesh matvec")
    ap.add_argument("--refactor", type=int, default=0, help="rehearsal: time a second factorisation")
    ap.add_argument("--interior", default="auto", help="velocity factorisation: auto (nested dissection), nested")
    ap.add_argument("--threads", type=int, default=16, help="rehearsal: host threads shared by the ranks")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    (rehearsal if args.mode == "rehearsal" else solo)(args)


if __name__ == "__main__":
    main()
