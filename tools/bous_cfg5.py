"""BASELINE cfg5: the element-partitioned Boussinesq coupler, 128 x 128 elements, P = 12 (2,362,369 nodes
per field, 9.45 M coupled DOFs), both solvers strip-partitioned over the ranks
(sem_amd.solvers.boussinesq.partitioned_coupler).  Times the coupled maps the Newton-Krylov iteration
calls (OpenMDAO/Boussinesq_SequentialCoupler.py:75-93 through the components' apply_nonlinear /
linearize / apply_linear), on host vectors as the coupler passes them, and the device part alone
(strip launches + interface exchange on device tensors).

  python tools/bous_cfg5.py                                   # one rank
  torchrun --nproc-per-node N tools/bous_cfg5.py              # N ranks, one GPU each, RCCL
  torchrun --nproc-per-node N tools/bous_cfg5.py --backend gloo   # N ranks on one GPU (rehearsal)
Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _timed(fn, reps, dev):
    ts = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=128)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--Ra", type=float, default=1e6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--exchange", default="allreduce", choices=["allreduce", "p2p"])
    args = ap.parse_args()
    if "RANK" not in os.environ:
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count() if args.backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    from sem_amd.solvers.boussinesq import partitioned_coupler
    Re, Pr = 1e3, 0.71
    t0 = time.perf_counter()
    c = partitioned_coupler(dist, 1.0, 1.0, Re, args.Ra, Pr, args.P, args.ne, args.ne, args.P, args.ne, args.ne,
                            exchange=args.exchange)
    setup = time.perf_counter() - t0
    r = np.random.default_rng(55)
    x, dx = r.uniform(-0.5, 0.5, c.DOF), r.uniform(-1, 1, c.DOF)
    c.residuals(x)
    c.linearize(x)
    c.jacobian_apply(dx)   # warm-up: graphs, caches
    out = {"config": f"cfg5 element-partitioned Boussinesq maps, {args.ne}x{args.ne} P={args.P}",
           "ranks": world, "backend": args.backend, "exchange": args.exchange, "DOF": int(c.DOF),
           "setup_s": setup}
    out["residuals_s"] = _timed(lambda: c.residuals(x), args.reps, dev)
    out["linearize_s"] = _timed(lambda: c.linearize(x), args.reps, dev)
    out["jacobian_apply_s"] = _timed(lambda: c.jacobian_apply(dx), args.reps, dev)
    # device part alone: this rank's strip tensors in, strip tensors out (launch + interface exchange)
    cd, ns = c.cd, c.ns
    n = ns._mesh.n_local
    loc = [torch.from_numpy(np.ascontiguousarray(ns._part.local(a))).to(dev) for a in np.split(x[c.Ncd:], 3)]
    T = torch.from_numpy(np.ascontiguousarray(cd._part.local(x[:c.Ncd]))).to(dev)
    out["ns_residuals_device_s"] = _timed(lambda: ns._get_residuals(*loc, T), max(args.reps, 20), dev)
    out["cd_residuals_device_s"] = _timed(lambda: cd._get_residuals(T, loc[0], loc[1]), max(args.reps, 20), dev)
    out["nodes_per_rank"] = int(n)
    if rank == 0:
        out["device"] = torch.cuda.get_device_name(dev)
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
