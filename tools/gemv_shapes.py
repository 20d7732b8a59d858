"""Streaming row GEMV (sem_gemv_rows, csrc/block_gemv.hip) on the strip solve's operator shapes, each operator read
once (several distinct copies cycled so nothing is served from the 256 MB MALL): the reduced-system rows Z
(2m x (G+1)m), the back substitution [X0 X1] (k m x 2m) and a sweep line's forward operator (m x 2m), m = 3,074
(cfg5), G = 8, k = 15.  HIP events around one graph of `reps` launches; bytes = the operator.

python tools/gemv_shapes.py [--m 3074 --G 8 --k 15]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=3074)
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--k", type=int, default=15)
    ap.add_argument("--reps", type=int, default=12)
    a = ap.parse_args()
    from sem_amd.solvers.velocity_solve import _gemv
    m = a.m
    shapes = {"Z (2m x (G+1)m)": (2 * m, (a.G + 1) * m), "X01 (k m x 2m)": (a.k * m, 2 * m),
              "sweep F (m x 2m)": (m, 2 * m)}
    out = {}
    for name, (M, K) in shapes.items():
        copies = max(2, int(3e9 // (8 * M * K)) + 1)
        As = [torch.rand((M, K), dtype=torch.float64, device="cuda") for _ in range(copies)]
        x = torch.rand(K, dtype=torch.float64, device="cuda")
        y = torch.empty(M, dtype=torch.float64, device="cuda")
        for A in As:
            _gemv(A, x, y)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
            for r in range(a.reps):
                _gemv(As[r % copies], x, y)
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
            best = min(best, e0.elapsed_time(e1) / a.reps)
        gb = 8.0 * M * K / 1e9
        out[name] = {"M": M, "K": K, "ms": best, "GB": gb, "TB_s": gb / best, "copies": copies}
        print(json.dumps({name: out[name]}), flush=True)
        del As, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
