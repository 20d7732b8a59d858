"""Micro-benchmark of the fused Navier-Stokes apply (sem_ns_apply, sem_amd/csrc/ns_apply.hip) in the three
forms the solvers launch -- the residual (_get_residuals: u, v, p, T in; ru, rv, rc out), the Schur
gradient (p in; ru, rv out in the line-interleaved [u | v] layout) and the Schur divergence (u, v
interleaved + p in; rc out) -- at cfg4 (48^2, P=8) and cfg5 (128^2, P=12).  Graph-replayed launches timed
with HIP events on the launch stream; algorithmic bytes = one read of every input vector and one write
of every output (fp64).

python tools/nsbench.py [--meshes 8:48,12:128] [--reps 200] [--kernels band,tile]
(--kernels: the band form (default) and the LDS-tile form, SEM_TUNE_NS_APPLY, A/B in one process)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--meshes", default="8:48,12:128")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--kernels", default="band")
    a = ap.parse_args()
    from sem_amd import _lib
    lib = _lib.load()
    from sem_amd.device import get_mesh
    dev = torch.device("cuda", 0)
    sides = _lib.SIDE_W | _lib.SIDE_E | _lib.SIDE_S | _lib.SIDE_N
    for spec in a.meshes.split(","):
        P, ne = map(int, spec.split(":"))
        m = get_mesh(P, ne, ne, 1.0 / ne, 1.0 / ne)
        N, NX, NY = m.n_local, m.NX, m.NY
        vec = lambda: torch.rand(N, dtype=torch.float64, device=dev) * 2 - 1  # noqa: E731
        u, v, p, T = (vec() for _ in range(4))
        du, dv, dp = (vec() for _ in range(3))
        jac = dict(juu=vec(), juv=vec(), jvu=vec(), jvv=vec())
        ru, rv, rc = (torch.empty_like(u) for _ in range(3))
        B = torch.rand((NX, 2 * NY), dtype=torch.float64, device=dev)
        # Sys = K + Re (u G_x + v G_y): the convecting velocity is the residual's own u, v (as the solver passes it)
        kw = dict(c_stiff=1.0, c_gradx=1e3, cu=u, c_grady=1e3, cv=v, dir_sides=sides, pin=N // 2)
        reps = a.reps if N < 1e6 else max(20, a.reps // 10)
        forms = {
            "residual": (lambda: m.ns_apply(u, v, p, ru, rv, rc, c_T=-1.4e3, T=T, pin_first=True, **kw), 7 * 8 * N),
            "dresidual": (lambda: m.ns_apply(du, dv, dp, ru, rv, rc, **kw, **jac), 12 * 8 * N),
            "schur_gradient": (lambda: m.ns_apply(None, None, p, B[:, :NY], B[:, NY:], dir_sides=sides, pin=N // 2),
                               3 * 8 * N),
            "schur_divergence": (lambda: m.ns_apply(B[:, :NY], B[:, NY:], p, rc=rc, c_div=-1.0, dir_sides=sides,
                                                    pin=N // 2), 4 * 8 * N),
        }
        for kern in a.kernels.split(","):
          _lib.check(lib.sem_set_tuning(_lib.TUNE_NS_APPLY, 1 if kern == "tile" else 0))
          for name, (fn, nbytes) in forms.items():
            us = timed(fn, reps)
            print(json.dumps({"mesh": f"{ne}x{ne} P={P}", "N": N, "kernel": kern, "form": name, "us_per_launch": us,
                              "bytes": nbytes, "GBps": nbytes / (us * 1e-6) / 1e9,
                              "frac_8TBps": nbytes / (us * 1e-6) / 8e12}), flush=True)
        _lib.check(lib.sem_set_tuning(_lib.TUNE_NS_APPLY, 0))
        del u, v, p, T, ru, rv, rc, B


if __name__ == "__main__":
    main()
