"""A short program for rocprofv3 counter passes over the nested-dissection velocity solve (tools/pmc_run.sh): the
cfg5 velocity Jacobian of a smooth linearisation factored once (tools/nd_probe.py's), then --solves eager solves.
The per-kernel HBM bytes of the solve's launches (FETCH_SIZE / WRITE_SIZE by grid size) set against the operator
bytes each step streams show whether any level re-reads its operators.

    tools/pmc_run.sh OUT -- python tools/nd_pmc_target.py --ne 128 --P 12 --solves 5
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=128)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--solves", type=int, default=5)
    ap.add_argument("--plan", default="", help="write the launch plan (grid size, operator bytes per step) here")
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    dev = torch.device("cuda", 0)
    ns = NavierStokesSolver(1.0, 1.0, 1e3, 1e6 / 0.71, args.P, args.ne, args.ne, mtol=1e-10, mtol_newton=1e-10,
                            iprint=[], velocity_graph=False)
    x, y = ns.points
    u0 = 1e-2 * np.sin(np.pi * x) * np.sin(2 * np.pi * y)
    v0 = -1e-2 * np.sin(2 * np.pi * x) * np.sin(np.pi * y)
    ns._get_residuals(u0, v0, np.zeros(ns.N), 0.5 - x)
    ns._calc_jacobians(u0, v0)
    vs = ns._velocity_solver()
    assert vs.interior == "nd"
    r = np.random.default_rng(5)
    bu, bv = (ns._dev(r.uniform(-1, 1, ns.N)) for _ in range(2))
    for _ in range(args.solves):
        vs.solve(bu, bv)
    torch.cuda.synchronize(dev)
    if args.plan:
        steps = []
        from sem_amd import _lib
        for k, (d, keep, sc, sp) in enumerate(vs._hip):
            if isinstance(d, _lib.SemLeafLaunch):
                steps.append({"step": k, "leaf": "split", "grid": d.nelem * 256, "op_bytes": vs._leafB.numel() * 8})
                continue
            dims = keep["dims"].cpu().numpy()
            steps.append({"step": k, "back": d.back, "form": d.form, "grid": d.ntiles * 256,
                          "op_bytes": int((dims[:, 0].astype(np.int64) * dims[:, 1]).sum() * 8),
                          "sparse_bytes": sp["coef"].numel() * 8 if sp else 0})
        with open(args.plan, "w") as f:
            json.dump(steps, f, indent=1)


if __name__ == "__main__":
    main()
