"""Timing of the dense kernels of the interface sweep's factorisation at cfg5's block size (m = 2 N_y =
3,074): one pivot-block inverse by each route (torch.linalg.inv; lu_factor + lu_solve against I;
rocSOLVER strided-batched getrf + getri with batch 1; lu_factor alone) beside one m^3 GEMM, to say where
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
    a = ap.parse_args()
    from sem_amd import linalg
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
    }
    for name, f in routes.items():
        f()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            f()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        print(json.dumps({"m": m, "route": name, "ms": round(ms, 3),
                          "tflops_2m3": round(2.0 * m ** 3 / (ms * 1e-3) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
