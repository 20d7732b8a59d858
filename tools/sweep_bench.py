"""HBM rate of the Krylov-basis sweep kernels (sem_basis_dot2, sem_basis_update) beside torch's
GEMV route, on a basis of k rows x n doubles (default: k = 1000, n = 263169, the 64^2 P=8 CD solve
mid-way through its Arnoldi process).  Algorithmic bytes: dot2 reads V and two vectors, update
reads V and reads + writes w."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--n", type=int, default=263169)
    args = ap.parse_args()
    from sem_amd.krylov import _DeviceSweeps
    k, n = args.k, args.n
    V = torch.rand((k + 1, n), dtype=torch.float64, device="cuda")
    a, b, w = (torch.rand(n, dtype=torch.float64, device="cuda") for _ in range(3))
    c = torch.rand(k, dtype=torch.float64, device="cuda")
    sw = _DeviceSweeps(V)
    Vk = V[:k]
    by_dot, by_upd = 8.0 * (k * n + 2 * n), 8.0 * (k * n + 2 * n)
    out = {"k": k, "n": n, "peak_GBs": 8000.0}
    for name, fn, by in (("dot2_hip", lambda: sw.dot2(k, a, b), by_dot),
                         ("dot2_torch_2gemv", lambda: (Vk @ a, Vk @ b), 8.0 * (2 * k * n + 2 * n)),
                         ("update_hip", lambda: sw.update(k, c, w), by_upd),
                         ("update_torch_gemv", lambda: w - Vk.T @ c, by_upd)):
        t = timed(fn)
        out[name] = {"us": t * 1e6, "GBs": by / t / 1e9, "frac": by / t / 1e9 / 8000.0}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
