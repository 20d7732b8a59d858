"""The block GEMVs of cfg5's interface sweep (block Thomas over the N_ex + 1 interface lines, m = 2 N_y =
3074 unknowns per line): torch's GEMV (rocBLAS) against sem_block_gemv (sem_amd/csrc/block_gemv.hip) on
one m x m and one m x 2m block, each timed as 100 launches in one hipGraph (HIP events on the launch
stream); bytes = the block (8 S m^2), read once.

python tools/gemv_probe.py [--m 3074]
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_us(fn, reps=100):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
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
    ap.add_argument("--m", type=int, default=3074)
    m = ap.parse_args().m
    from sem_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    lines = 4
    g = torch.rand((lines, m), dtype=torch.float64, device=dev)
    z = torch.zeros_like(g)
    for S in (1, 2):
        M = torch.rand((1, m, S * m), dtype=torch.float64, device=dev)
        rhs = torch.rand((S * m,), dtype=torch.float64, device=dev)
        out = torch.empty((m,), dtype=torch.float64, device=dev)
        t_torch = graph_us(lambda: torch.mv(M[0], rhs, out=out))
        xrow = torch.tensor([[1], [2]][:S], dtype=torch.int64, device=dev)
        yrow = torch.tensor([3], dtype=torch.int64, device=dev)
        srcs = (g, z)[:S] if S == 2 else (g,)
        P = C.c_void_p
        src = (P * S)(*(P(t.data_ptr()) for t in srcs))
        ld = (C.c_int64 * S)(*(t.stride(0) for t in srcs))

        def hip():
            st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            _lib.check(lib.sem_block_gemv(1, m, S, P(M.data_ptr()), src, ld, P(xrow.data_ptr()), P(z.data_ptr()),
                                          z.stride(0), P(yrow.data_ptr()), 0, st))
        t_hip = graph_us(hip)
        nbytes = 8.0 * S * m * m
        print(json.dumps({"m": m, "S": S, "bytes": nbytes, "torch_mv_us": t_torch, "torch_TBps": nbytes / t_torch / 1e6,
                          "sem_block_gemv_us": t_hip, "sem_TBps": nbytes / t_hip / 1e6}), flush=True)


if __name__ == "__main__":
    main()
