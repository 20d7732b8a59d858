"""In-process A/B of a libsemops kernel-selection knob (include/sem_ops.h enum sem_tune), set
through sem_set_tuning between captures (the library reads the environment only once).

python tools/ab_env.py --var SEM_BAND_CPOL --values 0,1,3 [--meshes 8:64,8:1024] [--rounds 5]
Each round times every value once (graph-replayed back-to-back CD applies, HIP events), so
clock and thermal drift spread over all values; prints the per-value median and min in us.
"""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import time_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--meshes", default="8:64,8:1024")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=0, help="applies per graph (0: 400 small / 20 large)")
    args = ap.parse_args()
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    vals = args.values.split(",")
    lib = _lib.load()
    knob = {"SEM_BAND_TILE": _lib.TUNE_BAND_TILE, "SEM_BAND_KP": _lib.TUNE_BAND_KP,
            "SEM_MFMA_TILE": _lib.TUNE_MFMA_TILE}[args.var]
    for spec in args.meshes.split(","):
        P, ne = (int(a) for a in spec.split(":"))
        mesh = get_mesh(P, ne, ne, 1.0 / ne, 1.0 / ne)
        N = mesh.n_local
        r = np.random.default_rng(0)
        T, u, v = (mesh.to_device(r.uniform(-1, 1, N)) for _ in range(3))
        y = torch.empty_like(T)
        kw = dict(c_stiff=1.0, c_gradx=40.0, cu=u, c_grady=40.0, cv=v, dir_mode=_lib.DIR_IDENTITY,
                  dir_sides=_lib.SIDE_W | _lib.SIDE_E)
        reps = args.reps or (400 if N < 4_000_000 else 20)
        ref = None
        res = {v_: [] for v_ in vals}
        for _ in range(args.rounds):
            for v_ in vals:
                val = int(v_)
                if knob == _lib.TUNE_BAND_KP:   # SEM_BAND_KP=0 means struct-only arguments (knob value -1)
                    val = -1 if val == 0 else 0
                _lib.check(lib.sem_set_tuning(knob, val))
                res[v_].append(time_graph(lambda: mesh.apply(T, y, **kw), reps))
                if ref is None:
                    ref = y.clone()
                elif not torch.equal(y, ref):
                    print(f"  {args.var}={v_}: RESULT DIFFERS", flush=True)
        for v_ in vals:
            med, mn = statistics.median(res[v_]), min(res[v_])
            print(f"P={P:2d} ne={ne:5d} N={N:9d} {args.var}={v_:>5s}: median {med:9.2f} us  min {mn:9.2f} us  "
                  f"{32.0 * N / med / 1e3:8.1f} GB/s", flush=True)
        _lib.check(lib.sem_set_tuning(knob, 0))


if __name__ == "__main__":
    main()
