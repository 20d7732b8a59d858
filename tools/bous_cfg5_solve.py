"""BASELINE cfg5 end to end: the Boussinesq coupler at 128 x 128 elements, P = 12, JNK from rest at the
given Ra (Ra continuation through --continuation).  One rank: the whole-mesh device coupler
(BoussinesqCoupler, the coupled vector on the device).  Several ranks: the element-partitioned coupler
(partitioned_coupler: both solvers strip-partitioned, the Newton updates element-partitioned too).

  python tools/bous_cfg5_solve.py --continuation 1e3 --Ra 1e4 [--ckpt DIR]          # one MI355X
  torchrun --nproc-per-node N tools/bous_cfg5_solve.py [--Ra 1e3]                  # RCCL, one GPU per rank
  torchrun --nproc-per-node N tools/bous_cfg5_solve.py --backend gloo              # N ranks on one GPU
Prints the Newton history and one JSON line per stage (rank 0).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=128)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--Ra", type=float, default=1e3)
    ap.add_argument("--mode", default="JNK")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--continuation", default="", help="Ra stages before --Ra (each starts from the last)")
    ap.add_argument("--out", default="")
    ap.add_argument("--ckpt", default="", help="directory for each finished stage's state (rank 0)")
    ap.add_argument("--interior", default="", help="velocity factorisation: auto (nested dissection) or nested")
    ap.add_argument("--x0", default="", help="start from a saved state (.npy of [T, u, v, p])")
    args = ap.parse_args()
    if "RANK" not in os.environ:
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29534")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count() if args.backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    if args.backend == "gloo" and world > 1:   # rehearsal: the ranks share the box's 16-CPU share
        torch.set_num_threads(max(1, 16 // world))
    import gc

    from sem_amd.solvers.boussinesq import BoussinesqCoupler, partitioned_coupler
    Re, Pr = 1e3, 0.71
    x, stages = (np.load(args.x0) if args.x0 else None), []
    for Ra in [float(r) for r in args.continuation.split(",") if r] + [args.Ra]:
        if world == 1:
            c = BoussinesqCoupler(1.0, 1.0, Re, Ra, Pr, args.P, args.ne, args.ne, args.P, args.ne, args.ne,
                                  mode=args.mode, iprint=2)
        else:
            c = partitioned_coupler(dist, 1.0, 1.0, Re, Ra, Pr, args.P, args.ne, args.ne, args.P, args.ne, args.ne,
                                    mode=args.mode, iprint=2 if rank == 0 else 0)
        if args.interior:   # A/B of the velocity factorisation (NavierStokesSolver velocity_interior)
            c.ns._velocity_interior = args.interior
        if rank == 0:   # progress lines from the Schur / CD Krylov solves, and the factorisation times
            c.ns._progress, c.cd._progress = 250, 250
            c.ns._iprint = ["LU_suc"]
        t0 = time.perf_counter()
        T, u, v, p = c.solve(x)
        dt = time.perf_counter() - t0
        x = np.concatenate([T, u, v, p])
        res = float(np.linalg.norm(c.residuals(x)))   # collective
        if rank == 0 and args.ckpt:
            os.makedirs(args.ckpt, exist_ok=True)
            np.save(os.path.join(args.ckpt, f"cfg5_{Ra:g}.npy"), x)
        if rank == 0:
            s = np.linspace(0.0, 1.0, 1001)
            um = np.asarray(c.ns._get_interpol(u, np.meshgrid([0.5], s, indexing="ij")))[0] * Re * Pr
            vm = np.asarray(c.ns._get_interpol(v, np.meshgrid(s, [0.5], indexing="ij")))[:, 0] * Re * Pr
            st = {"Ra": Ra, "newton_iters": c.iterations, "seconds": dt, "timing": c.timing, "calls": c.calls,
                  "u_max_midline": float(um.max()), "u_max_y": float(s[um.argmax()]),
                  "v_max_midline": float(vm.max()), "v_max_x": float(s[vm.argmax()]),
                  "residual_2norm": res, "tolerance": float(c.atol_nonlin)}
            stages.append(st)
            print(json.dumps(st), flush=True)
        del c
        gc.collect()
        torch.cuda.empty_cache()
    if rank == 0:
        out = {"config": f"Boussinesq {args.mode} Ra={args.Ra:g}, {args.ne}x{args.ne} P={args.P}"
                         + (", element-partitioned" if world > 1 else ", whole mesh on one GPU"),
               "ranks": world, "backend": args.backend, "DOF": int(x.size), "stages": stages,
               "device": torch.cuda.get_device_name(dev)}
        print(json.dumps(out), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(out, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
