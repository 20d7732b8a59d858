"""Timing of the dense kernels of the interface sweep's factorisation at cfg5's block size (m = 2 N_y =
3,074): one pivot-block inverse by each route (torch.linalg.inv; lu_factor + lu_solve against I;
rocSOLVER strided-batched getrf + getri with batch 1; lu_factor alone; the GEMM-recursive block inverse
at three leaf sizes, and the checked pivot_inverse) beside one m^3 GEMM, to say where
the 129 sequential block-Thomas steps of the cfg5 factorisation spend their time.

python tools/pivot_probe.py [--m 3074] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=3074)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    from sem_amd import linalg
    from sem_amd.solvers.velocity_solve import pivot_inverse
    dev = torch.device("cuda", 0)
    m = a.m
    g = torch.Generator(device=dev).manual_seed(1)
    A = torch.rand((m, m), dtype=torch.float64, device=dev, generator=g) - 0.5 + m ** 0.5 * torch.eye(m, device=dev,
                                                                                                        dtype=torch.float64)
    B = torch.rand((m, m), dtype=torch.float64, device=dev, generator=g)
    I = torch.eye(m, dtype=torch.float64, device=dev)
    routes = {
        "gemm": lambda: A @ B,
        "inv": lambda: torch.linalg.inv(A),
        "lu_factor": lambda: torch.linalg.lu_factor(A),
        "lu_factor+lu_solve(I)": lambda: torch.linalg.lu_solve(*torch.linalg.lu_factor(A), I),
        "rocsolver_strided_b1": lambda: linalg.strided_inverse(A[None])[0],
        "solve(A, B)": lambda: torch.linalg.solve(A, B),
        "block_inverse_b32": lambda: linalg.block_inverse(A, base=32),
        "block_inverse_b64": lambda: linalg.block_inverse(A, base=64),
        "block_inverse_b128": lambda: linalg.block_inverse(A, base=128),
        "block_inverse_b256": lambda: linalg.block_inverse(A, base=256),
        "block_inverse_b512": lambda: linalg.block_inverse(A, base=512),
        "pivot_inverse(block+check)": lambda: pivot_inverse(A),
    }
    if a.profile:
        leaf_times()
        profile(A)
        return
    for name, f in routes.items():
        f()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            f()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        out = {"m": m, "route": name, "ms": round(ms, 3), "tflops_2m3": round(2.0 * m ** 3 / (ms * 1e-3) / 1e12, 2)}
        if name != "gemm" and not name.startswith("lu_factor") and name != "solve(A, B)":
            X = f()
            X = X[0] if isinstance(X, tuple) else X
            E = A @ X - I
            out["max_abs_AX_minus_I"] = float(E.abs().max())
        print(json.dumps(out), flush=True)


def leaf_times():
    """Per-launch time of the Gauss-Jordan leaf kernel against n (a + b n: b = one elimination step),
    200 back-to-back launches in one graph, HIP events."""
    from sem_amd import linalg
    dev = torch.device("cuda", 0)
    for n in (8, 16, 32, 48, 64):
        A = torch.rand((n, n), dtype=torch.float64, device=dev) + n * torch.eye(n, dtype=torch.float64, device=dev)
        X = torch.empty_like(A)
        linalg.small_inverse_into(A, X)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
            for _ in range(200):
                linalg.small_inverse_into(A, X)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"leaf_n": n, "us_per_launch": round(e0.elapsed_time(e1) * 1e3 / 200, 2)}), flush=True)


def profile(A):
    """Kernel-time breakdown of one block_inverse call (torch profiler, device time per kernel name)."""
    from torch.profiler import profile as prof, ProfilerActivity
    from sem_amd import linalg
    for base in (64, 256):
        linalg.block_inverse(A, base=base)
        torch.cuda.synchronize()
        with prof(activities=[ProfilerActivity.CUDA]) as p:
            linalg.block_inverse(A, base=base)
            torch.cuda.synchronize()
        print(f"block_inverse base {base}", flush=True)
        print(p.key_averages().table(sort_by="cuda_time_total", row_limit=12), flush=True)


if __name__ == "__main__":
    main()
