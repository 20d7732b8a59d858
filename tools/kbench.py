"""Kernel micro-benchmark: fused CD apply (32 B/DOF algorithmic) at several meshes.

python tools/kbench.py [--algo 0|1|2] [--reps 200]
Times graph-replayed back-to-back applies with HIP events; prints one line per mesh.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def time_graph(fn, reps):
    for _ in range(3):
        fn()
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
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


STAMP_BUF = None
if os.environ.get("SEM_DIAG_BUF") == "auto":  # allocate the stamp buffer before libsemops reads the variable
    STAMP_BUF = torch.zeros(1 << 22, dtype=torch.int64, device="cuda")
    os.environ["SEM_DIAG_BUF"] = str(STAMP_BUF.data_ptr())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--meshes", default="8:64,12:128,8:256,8:1024,4:512")
    ap.add_argument("--floor", action="store_true", help="also time torch.addcmul (same 32 B/DOF traffic)")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic: per-wave phase stamps of one apply (needs SEM_DIAG=8 and SEM_DIAG_BUF)")
    ap.add_argument("--nstamps", type=int, default=7, help="stamps per wave written by the kernel")
    ap.add_argument("--roles", default="", help="wave roles by slot within a workgroup, e.g. X:0-3,Y:4-7,E:8")
    ap.add_argument("--stride", type=int, default=8, help="stamp slots per wave (band kernel: 16)")
    ap.add_argument("--tiles-x", type=int, default=32)
    ap.add_argument("--tiles-y", type=int, default=8)
    ap.add_argument("--dss", type=int, default=0,
                    help="FETCH_SIZE calibration: time sem_dss on an ne x ne, P=8 element array (8-byte loads, "
                         "reads exactly ne^2*81*8 bytes)")
    a = ap.parse_args()
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    dev = torch.device("cuda", 0)
    if a.stamps:
        import numpy as np
        buf = STAMP_BUF
        P, ne = map(int, a.meshes.split(",")[0].split(":"))
        m = get_mesh(P, ne, ne, 1.0 / ne, 1.0 / ne)
        T, u, v = (torch.rand(m.n_local, dtype=torch.float64, device=dev) for _ in range(3))
        y = torch.empty_like(T)
        kw = dict(c_stiff=1.0, c_gradx=40.0, cu=u, c_grady=40.0, cv=v, dir_mode=_lib.DIR_IDENTITY,
                  dir_sides=_lib.SIDE_W | _lib.SIDE_E, algo=a.algo)
        for _ in range(20):
            m.apply(T, y, **kw)
        buf.zero_()
        torch.cuda.synchronize()
        m.apply(T, y, **kw)
        torch.cuda.synchronize()
        st = buf.cpu().numpy().reshape(-1, a.stride).astype(np.int64)
        slot = np.arange(len(st))
        keep = st[:, 0] > 0
        st, slot = st[keep], slot[keep]
        t0 = st[:, 0].min()
        ns = int(a.nstamps)
        print(f"{m.kernel_name(a.algo)}: {len(st)} waves; times in shader cycles relative to the first wave start")
        roles = {"all": np.ones(len(st), bool)}
        if a.roles:  # e.g. "X:0-3,Y:4-7,E:8" wave slots within a workgroup of NW waves
            nw = max(int(r.split(":")[1].split("-")[-1]) for r in a.roles.split(",")) + 1
            for r in a.roles.split(","):
                nm, rg = r.split(":")
                lo, hi = (int(x) for x in (rg.split("-") + rg.split("-"))[:2]) if "-" in rg else (int(rg), int(rg))
                roles[nm] = ((slot % nw) >= lo) & ((slot % nw) <= hi)
        for nm, sel in roles.items():
            sr = st[sel]
            if len(sr) == 0:
                continue
            line = " ".join(f"s{k}:{int(np.median(sr[:, k] - sr[:, 0])):6d}" for k in range(1, ns))
            print(f"  {nm:4s} ({len(sr):5d} waves) med since own start: {line}; start med {int(np.median(sr[:, 0] - t0))}")
        for k in range(1, ns):
            d = st[:, k] - st[:, k - 1]
            print(f"  phase s{k-1}->s{k}: med {int(np.median(d)):7d}  p90 {int(np.percentile(d, 90)):7d}")
        if a.stride >= 16 and (st[:, 10] > 0).any():   # band kernel slot 10: epilogue values formed, before the stores
            d1, d2 = st[:, 10] - st[:, 4], st[:, 5] - st[:, 10]
            print(f"  epilogue: s4->values formed med {int(np.median(d1))} p90 {int(np.percentile(d1, 90))}; "
                  f"stores issued med {int(np.median(d2))} p90 {int(np.percentile(d2, 90))}")
        last = ns - 1
        # per-XCD view (each XCD has its own clock): dispatch ramp, wave span, active window
        xcc = st[:, 7] & 0xF
        hw = st[:, 7] >> 8  # HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]
        cu = (xcc << 8) | ((hw >> 8) & 0xFF)
        win, ramp = [], []
        for c in sorted(set(cu.tolist())):
            sc = st[cu == c]
            win.append(sc[:, last].max() - sc[:, 0].min())
            ramp.append(sc[:, 0].max() - sc[:, 0].min())
        print(f"  per CU ({len(win)} CUs): active window med {int(np.median(win))} max {int(np.max(win))}; "
              f"start ramp med {int(np.median(ramp))} max {int(np.max(ramp))}; waves/CU {len(st) / len(win):.1f}")
        if a.stride >= 10:  # per-tile times on the chip-wide realtime clock (10 ns ticks), by tile class
            nw = max(int(r.split(":")[1].split("-")[-1]) for r in a.roles.split(",")) + 1 if a.roles else 1
            blk = slot // nw
            r0 = st[:, 8].min()
            beg, ends, cls = [], [], []
            for bidx in np.unique(blk):
                sb = st[blk == bidx]
                beg.append((sb[:, 8].min() - r0) * 10)
                ends.append((sb[:, 9].max() - r0) * 10)
                tx, ty = divmod(int(sb[0, 6]), a.tiles_y)
                cls.append(("X" if tx == a.tiles_x - 1 else "") + ("Y" if ty == a.tiles_y - 1 else "") or "I")
            beg, ends, cls = np.array(beg), np.array(ends), np.array(cls)
            print(f"  realtime (ns): workgroup start med {int(np.median(beg))} max {int(beg.max())}; "
                  f"end med {int(np.median(ends))} p90 {int(np.percentile(ends, 90))} max {int(ends.max())}")
            for c in sorted(set(cls.tolist())):
                e, b0 = ends[cls == c], beg[cls == c]
                print(f"  tiles {c:2s}: n {len(e):4d}  start med {int(np.median(b0)):5d}  end med {int(np.median(e)):5d}"
                      f" p90 {int(np.percentile(e, 90)):5d} max {int(e.max()):5d}  span med {int(np.median(e - b0))}")
        for x in sorted(set(xcc.tolist())):
            sx = st[xcc == x]
            s0 = sx[:, 0].min()
            print(f"  xcd {x}: waves {len(sx):5d}  last start {sx[:, 0].max() - s0:7d}  first end {sx[:, last].min() - s0:7d}"
                  f"  last end {sx[:, last].max() - s0:7d}  med span {int(np.median(sx[:, last] - sx[:, 0])):6d}")
        return
    if a.dss:
        m = get_mesh(8, a.dss, a.dss, 1.0 / a.dss, 1.0 / a.dss)
        ae = torch.rand((a.dss, a.dss, 9, 9), dtype=torch.float64, device=dev)
        out = torch.empty(m.n_local, dtype=torch.float64, device=dev)
        t = time_graph(lambda: m.dss(ae, out), 20)
        rb, wb = ae.numel() * 8, out.numel() * 8
        print(f"dss ne={a.dss}: {t:9.2f} us  reads {rb / 1e6:.1f} MB  writes {wb / 1e6:.1f} MB  "
              f"{(rb + wb) / (t * 1e-6) / 1e9:7.1f} GB/s", flush=True)
        return
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
        if a.floor:
            fl = time_graph(lambda: torch.addcmul(v, T, u, out=y), reps)
            print(f"    floor (torch.addcmul, 3 reads + 1 write): {fl:9.2f} us  {32.0 * N / (fl * 1e-6) / 1e9:7.1f} GB/s",
                  flush=True)
        del T, u, v, y, g


if __name__ == "__main__":
    main()
