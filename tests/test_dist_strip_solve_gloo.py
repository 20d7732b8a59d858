"""World-size 1/2/3/8 gloo tests (CPU) of the element-partitioned condensed direct solve
(sem_amd/solvers/strip_solve.py, StripLineSolver): each rank factors its strip's pieces -- the oracle
Jacobian's (NavierStokes_Solver.py:176-183, or the CD operator ConvectionDiffusion_Solver.py:104-121),
restricted to the strip, a shared interface line's own block held by its right owner -- eliminates its
interior interface lines, and the ranks solve the reduced system over the strip-boundary lines together.
The solution on every rank's lines equals SciPy's sparse solve of the whole Jacobian."""
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


def strip_pieces(pcs, P, bounds, rank):
    """The rank's strip of whole-mesh pieces (tests/velocity_blocks.extract layout): its columns' pieces,
    its lines' interface blocks, the right line's block zero when a strip to the right owns it."""
    eb, ee = bounds[rank], bounds[rank + 1]
    nex = bounds[-1]
    out = {k: pcs[k][eb:ee].copy() for k in ("AII", "aIB", "aBI", "E", "F")}
    out["D"] = pcs["D"][eb:ee + 1].copy()
    if ee < nex:
        out["D"][-1] = 0.0
    return out


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
        from velocity_blocks import extract, oracle_cd_jacobian, oracle_velocity_jacobian
        from sem_amd.parallel import StripPartition
        from sem_amd.solvers.strip_solve import StripLineSolver
        P, nex, ney, Re, ncomp, blocklu = case
        if ncomp == 2:
            ref, _, _ = oracle_velocity_jacobian(P, nex, ney, Re, seed=P * 10 + nex)
            J = ref.Jvelo
        else:
            ref, J, _, _ = oracle_cd_jacobian(P, nex, ney, Re, seed=P + nex)
        pcs = extract(J.toarray(), P, nex, ney, ncomp=ncomp)
        part = StripPartition(nex, world)
        vs = StripLineSolver(P, nex, ney, "cpu", part.bounds, rank, dist, ncomp=ncomp)
        if blocklu:
            vs.edge_dense_max = 0
        sp_ = {k: torch.as_tensor(v) for k, v in strip_pieces(pcs, P, part.bounds, rank).items()}
        vs.factor_condensed(None, pieces=vs.condense_dense(sp_.pop("AII")), line=sp_)
        NY, N = ney * P + 1, (nex * P + 1) * (ney * P + 1)
        r = np.random.default_rng(17)
        b = r.uniform(-1, 1, ncomp * N)
        want = spla.spsolve(J.tocsc(), b)
        eb, ee = part.bounds[rank], part.bounds[rank + 1]
        sl = slice(eb * P * NY, (ee * P + 1) * NY)
        comps = [b[c * N:(c + 1) * N][sl] for c in range(ncomp)]
        if ncomp == 2:
            got = vs.solve(torch.as_tensor(comps[0]), torch.as_tensor(comps[1]))
        else:
            got = (vs.solve1(torch.as_tensor(comps[0])),)
        err = max(np.abs(g.numpy() - want[c * N:(c + 1) * N][sl]).max() for c, g in enumerate(got))
        q.put((rank, err / np.abs(want).max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [
    (1, (4, 3, 2, 300.0, 2, False)),
    (2, (4, 4, 3, 300.0, 2, False)),    # two columns per strip: one interior interface line each
    (2, (3, 2, 4, 100.0, 2, True)),     # one column per strip: no interior line; block-LU edge inverses
    (3, (4, 7, 2, 700.0, 2, False)),    # uneven strips (3, 2, 2 columns)
    (2, (3, 9, 2, 300.0, 2, False)),    # strips of 5 and 4 columns: the two-ended interior sweep, X0 / X1 from its factors
    (3, (5, 6, 3, 40.0, 1, False)),     # the one-component (CD) operator
    # cfg5's world size: 8 ranks over 11 columns (strips of 2, 2, 2, 1, 1, 1, 1, 1 columns:
    # uneven, one-column strips with no interior line), and the CD operator over 9 columns (2, 1 x 7)
    (8, (4, 11, 2, 300.0, 2, False)),
    (8, (3, 9, 3, 40.0, 1, True)),
])
def test_strip_line_solver_gloo(world, case):
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
