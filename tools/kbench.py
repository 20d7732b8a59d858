"""Kernel micro-benchmark: fused CD apply (32 B/DOF algorithmic) at several meshes.

python tools/kbench.py [--algo 0|1|2] [--reps 200]
Times graph-replayed back-to-back applies with HIP events; prints one line per mesh.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--meshes", default="8:64,12:128,8:256,8:1024,4:512")
    a = ap.parse_args()
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    dev = torch.device("cuda", 0)
    for spec in a.meshes.split(","):
        P, ne = map(int, spec.split(":"))
        m = get_mesh(P, ne, ne, 1.0 / ne, 1.0 / ne)
        N = m.n_local
        T, u, v = (torch.rand(N, dtype=torch.float64, device=dev) for _ in range(3))
        y = torch.empty_like(T)
        kw = dict(c_stiff=1.0, c_gradx=40.0, cu=u, c_grady=40.0, cv=v, dir_mode=_lib.DIR_IDENTITY,
                  dir_sides=_lib.SIDE_W | _lib.SIDE_E, algo=a.algo)
        reps = a.reps if N < 5e6 else max(10, a.reps // 20)
        for _ in range(5):
            m.apply(T, y, **kw)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                m.apply(T, y, **kw)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps * 1e3)
        gbs = 32.0 * N / (best * 1e-6) / 1e9
        print(f"P={P:2d} ne={ne:5d} N={N:10d} algo={a.algo}: {best:9.2f} us/apply  {N / best / 1e3:9.3f} GDOF/s"
              f"  {gbs:7.1f} GB/s ({gbs / 8000 * 100:5.1f}% of 8 TB/s)", flush=True)
        del T, u, v, y, g


if __name__ == "__main__":
    main()
