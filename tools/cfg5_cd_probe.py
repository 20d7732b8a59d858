"""cfg5's convection-diffusion update on one MI355X (the whole-mesh counterpart rank 0 runs for the
element-partitioned coupler, partition_update="central"): 128 x 128, P = 12, Pe = Re Pr = 710, at the
coupled solve's first linearisation (fluid at rest) and at a seeded velocity field.  Reports the
column-chunked condensed factorisation, the relative residual of its solve through the fused Jacobian
apply, and the preconditioned GMRES update.

python tools/cfg5_cd_probe.py [--ne 128 --P 12]
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
    args = ap.parse_args()
    from sem_amd.solvers import ConvectionDiffusionSolver
    dev = torch.device("cuda", 0)
    cd = ConvectionDiffusionSolver(1.0, 1.0, 710.0, args.P, args.ne, args.ne, T_W=0.5, T_E=-0.5, mtol=1e-13)
    cd._progress = 50
    N = cd.N
    r = np.random.default_rng(3)
    for name, (u, v) in (("rest", (np.zeros(N), np.zeros(N))),
                         ("seeded", (0.01 * r.uniform(-1, 1, N), 0.01 * r.uniform(-1, 1, N)))):
        res = cd._get_residuals(np.zeros(N), u, v)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        vs = cd._jacobian_solver()
        torch.cuda.synchronize(dev)
        out = {"case": name, "N": N, "factor_s": time.perf_counter() - t0,
               "chunked": vs.interior_bytes() > (24 << 30)}
        b = cd._dev(r.uniform(-1, 1, N))
        x = vs.solve1(b)
        jx = cd._get_dresiduals(x)
        out["solve_rel_residual"] = float((jx - b).abs().max() / b.abs().max())
        vs.hip_nested = False
        x2 = vs._solve_lines(b.view(vs.NX, vs.m).clone()).reshape(-1)
        vs.hip_nested = True
        out["hip_vs_torch_nested"] = float((x2 - x).abs().max() / x.abs().max())
        print(json.dumps(out), flush=True)
        t0 = time.perf_counter()
        cd._get_update(-res)
        out["update_s"], out["update_matvecs"] = time.perf_counter() - t0, cd.matvecs
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
