"""cfg5's Navier-Stokes update on one MI355X (the whole-mesh counterpart rank 0 runs for the
element-partitioned coupler): 128 x 128 elements, P = 12, Re = 1e3, Gr = Ra / Pr at Ra = 1e6, linearised
at the coupled solve's starting state (fluid at rest, conduction temperature T = 1/2 - x).  Reports the
column-chunked velocity factorisation (time, peak device memory), the velocity solve (time, relative
residual of J x = b through the fused Jacobian apply) and one Newton update (_get_update: Schur Krylov
solve around the velocity solve) at the given tolerance.

python tools/cfg5_ns_probe.py [--ne 128 --P 12 --mtol 1e-10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=128)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--Ra", type=float, default=1e6)
    ap.add_argument("--mtol", type=float, default=1e-10)
    ap.add_argument("--update", type=int, default=1)
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    Re, Pr = 1e3, 0.71
    dev = torch.device("cuda", 0)
    ns = NavierStokesSolver(1.0, 1.0, Re, args.Ra / Pr, args.P, args.ne, args.ne, mtol=args.mtol, mtol_newton=args.mtol,
                            iprint=[])
    ns._progress = 250
    N = ns.N
    z = np.zeros(N)
    T = 0.5 - ns.points[0]
    out = {"config": f"cfg5 NS update, {args.ne}x{args.ne} P={args.P}, Ra={args.Ra:g}", "N": N}
    res = ns._get_residuals(z, z, z, T)
    ns._calc_jacobians(z, z)
    vs_tmp = None
    torch.cuda.synchronize(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    t0 = time.perf_counter()
    vs = ns._velocity_solver()
    torch.cuda.synchronize(dev)
    out["factor_s"] = time.perf_counter() - t0
    out["factor_peak_GB"] = torch.cuda.max_memory_allocated(dev) / 1e9
    out["interior_dense_GB_one_shot"] = vs.interior_bytes() / 1e9
    out["resident_GB"] = torch.cuda.memory_allocated(dev) / 1e9
    if vs.timing:   # SEM_PROFILE_FACTOR=1
        out["factor_phases_s"] = vs.timing
    print(json.dumps(out), flush=True)
    r = np.random.default_rng(7)
    bu, bv = (ns._dev(r.uniform(-1, 1, N)) for _ in range(2))
    xu, xv = vs.solve(bu, bv)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(5):
        xu, xv = vs.solve(bu, bv)
    torch.cuda.synchronize(dev)
    out["velocity_solve_ms"] = (time.perf_counter() - t0) / 5 * 1e3
    ju, jv, _ = ns._get_dresiduals(xu, xv, torch.zeros_like(xu))
    out["velocity_solve_rel_residual"] = float(max((ju - bu).abs().max(), (jv - bv).abs().max()) /
                                             max(bu.abs().max(), bv.abs().max()))
    print(json.dumps(out), flush=True)
    del vs_tmp
    if args.update:
        t0 = time.perf_counter()
        du, dv, dp = ns._get_update(-res[0], -res[1], -res[2])
        torch.cuda.synchronize(dev)
        out["update_s"] = time.perf_counter() - t0
        out["schur_matvecs"] = ns.schur_matvecs
        dru, drv, drc = ns._get_dresiduals(du, dv, dp)
        rr = np.sqrt(sum(float(np.sum((a + b) ** 2)) for a, b in zip((dru, drv, drc), res)))
        out["update_residual_2norm"] = rr
        out["update_tolerance"] = args.mtol * np.sqrt(N)
        out["peak_GB"] = torch.cuda.max_memory_allocated(dev) / 1e9
    out["device"] = torch.cuda.get_device_name(dev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
