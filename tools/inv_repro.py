"""Standalone reproducer for the batched-inverse failure seen in round 2: the
one-component condensation at P = 12 solved with relative residual 22-98 when its element-interior
blocks (121 x 121) were inverted in one batched call, and to 3e-13 in smaller batches.

This probe takes the condensation out of the picture: seeded, well-conditioned, contiguous blocks
(U(-1, 1) + n I) go straight into torch.linalg.inv (rocSOLVER getrf + getri batched), and each block is
checked through max |A X - I| relative to |A|max |X|max.  It also runs the same blocks through
lu_factor + lu_solve against the identity and torch.linalg.solve, and repeats the batched call on a
strided (non-contiguous) view, to separate a library fault from a caller-side cause.

python tools/inv_repro.py [--n 121,242] [--batches 64,128,256,384,512,1024,4096]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel_residual(A, X):
    E = A @ X
    E.diagonal(dim1=-2, dim2=-1).sub_(1.0)
    scale = A.abs().amax(dim=(-2, -1)) * X.abs().amax(dim=(-2, -1))
    return E.abs().amax(dim=(-2, -1)) / scale


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="121,242")
    ap.add_argument("--batches", default="64,128,256,384,512,1024,4096,16384")
    ap.add_argument("--seed", type=int, default=2024)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(args.seed)
    from sem_amd import linalg
    for n in (int(s) for s in args.n.split(",")):
        eye = torch.eye(n, dtype=torch.float64, device=dev)
        for nb in (int(s) for s in args.batches.split(",")):
            A = (torch.rand((nb, n, n), dtype=torch.float64, device=dev, generator=g) * 2 - 1) + n * eye
            out = {"n": n, "batch": nb}
            for name, f in (("inv", torch.linalg.inv),
                            ("inv_ex", lambda a: torch.linalg.inv_ex(a)[0]),
                            ("lu_solve", lambda a: torch.linalg.lu_solve(*torch.linalg.lu_factor(a),
                                                                         eye.expand_as(a))),
                            ("solve", lambda a: torch.linalg.solve(a, eye.expand_as(a))),
                            ("rocsolver_strided", lambda a: linalg.strided_inverse(a)[0])):
                try:
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    X = f(A)
                    torch.cuda.synchronize(dev)
                    ms = (time.perf_counter() - t0) * 1e3
                except RuntimeError as e:      # e.g. HIPBLAS_STATUS_ALLOC_FAILED in getrfBatched
                    out[name] = {"error": str(e).splitlines()[0][:160]}
                    continue
                r = rel_residual(A, X)
                bad = int((r > 1e-10).sum())
                out[name] = {"max_rel_residual": float(r.max()), "bad_blocks": bad, "ms": round(ms, 2),
                             "gflops": round(2.0 * nb * n ** 3 / (ms * 1e-3) / 1e9, 1),
                             "first_bad": int(torch.nonzero(r > 1e-10)[0, 0]) if bad else -1}
            # a strided view of twice the batch (every other block): the caller-side layout question
            A2 = torch.empty((2 * nb, n, n), dtype=torch.float64, device=dev)
            A2[0::2] = A
            A2[1::2] = eye
            try:
                X = torch.linalg.inv(A2[0::2])
                out["inv_strided_view"] = {"max_rel_residual": float(rel_residual(A, X).max()),
                                           "bad_blocks": int((rel_residual(A, X) > 1e-10).sum())}
            except RuntimeError as e:
                out["inv_strided_view"] = {"error": str(e).splitlines()[0][:160]}
            print(json.dumps(out), flush=True)
            del A, A2
            torch.cuda.empty_cache()
    print(json.dumps({"device": torch.cuda.get_device_name(dev), "torch": torch.__version__,
                      "hip": torch.version.hip}), flush=True)


if __name__ == "__main__":
    main()
