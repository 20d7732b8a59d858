"""In-process A/B of the fused apply between two builds of libsemops (e.g. this tree against a previous
round's sources built into another directory), alternating rounds so clocks and box drift hit both alike.

    python tools/ab_lib.py --libs sem_amd/lib/libsemops.so,sem_amd/lib_ab/r05/libsemops.so --meshes 8:64,8:1024

Each library is loaded with ctypes under its own handle (RTLD_LOCAL: separate kernels, separate host stubs);
sem_create / sem_apply are called through the ABI structs of sem_amd._lib (sem_apply_desc is unchanged across
ABI 12 -> 13).  The apply is the bench's CD operator (K + Pe (u Gx + v Gy), Dirichlet W/E rows; --lap: K only);
per-launch device time = graph of `reps` back-to-back applies / reps, median over `rounds` alternations.
Results are also compared bitwise (the two builds may differ in rounding: the max relative difference is printed).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from sem_amd import _lib
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--meshes", default="8:64,8:1024")
    ap.add_argument("--reps", type=int, default=0, help="applies per graph (0: 1000 on small meshes, 20 on large)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--lap", type=int, default=0)
    ap.add_argument("--algo", type=int, default=0, help="sem_apply_desc.algo (0 AUTO = band, 2 = MFMA)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    libs = []
    for p in a.libs.split(","):
        lib = C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL)
        lib.sem_create.restype = C.c_int
        lib.sem_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_int,
                                   C.POINTER(C.c_void_p)]
        lib.sem_apply.restype = C.c_int
        lib.sem_apply.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.sem_build_id.restype = C.c_char_p
        libs.append((p, lib))
    out = []
    for spec in a.meshes.split(","):
        P, ne = map(int, spec.split(":"))
        d = 1.0 / ne
        N = (ne * P + 1) ** 2
        g = torch.Generator(device=dev).manual_seed(2024)
        T, u, v = (torch.rand(N, dtype=torch.float64, device=dev, generator=g) * 2 - 1 for _ in range(3))
        ys = []
        fns = []
        for p, lib in libs:
            h = C.c_void_p()
            st = lib.sem_create(P, ne, ne, d, d, 0, ne, 0, C.byref(h))
            assert st == 0, (p, st)
            y = torch.empty_like(T)
            if a.lap:
                desc = _lib.SemApplyDesc(0.0, 1.0, 0.0, 0.0, None, None, 0.0, None, None, None, None, 0.0, 0, None, None,
                                         0, a.algo, 0, 0)
            else:
                desc = _lib.SemApplyDesc(0.0, 1.0, 40.0, 40.0, u.data_ptr(), v.data_ptr(), 0.0, None, None, None, None,
                                         0.0, _lib.DIR_IDENTITY, None, None, _lib.SIDE_W | _lib.SIDE_E, a.algo, 0, 0)

            def fn(lib=lib, h=h, desc=desc, y=y):
                s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
                st = lib.sem_apply(h, C.addressof(desc), T.data_ptr(), y.data_ptr(), s)
                assert st == 0, st
            fn()
            ys.append(y)
            fns.append(fn)
        torch.cuda.synchronize(dev)
        diff = float(((ys[0] - ys[1]).abs().max() / ys[1].abs().max()).item()) if len(ys) > 1 else 0.0
        reps = a.reps or (1000 if N < 4_000_000 else 20)
        graphs = []
        for fn in fns:
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s), torch.cuda.graph(gr, stream=s):
                for _ in range(reps):
                    fn()
            torch.cuda.current_stream(dev).wait_stream(s)
            gr.replay()
            graphs.append(gr)
        torch.cuda.synchronize(dev)
        ts = [[] for _ in graphs]
        for _ in range(a.rounds):
            for i, gr in enumerate(graphs):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gr.replay()
                e1.record()
                torch.cuda.synchronize(dev)
                ts[i].append(e0.elapsed_time(e1) * 1e3 / reps)
        rec = {"P": P, "ne": ne, "N": N, "lap": bool(a.lap), "algo": a.algo, "reps": reps, "max_rel_diff": diff,
               "us": {os.path.relpath(p, ROOT): float(np.median(t)) for (p, _), t in zip(libs, ts)},
               "us_all": {os.path.relpath(p, ROOT): [round(x, 3) for x in t] for (p, _), t in zip(libs, ts)}}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del graphs
    if a.out:
        with open(a.out, "a") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
