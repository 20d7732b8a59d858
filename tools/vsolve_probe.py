"""Roofline of the NS velocity solve (the inner solve of every Schur-complement matvec,
NavierStokes_Solver.py:189-203) at a given mesh: factor once, then time `--solves` graph-replayed solves
with HIP events, and account the algorithmic bytes one solve reads and writes, factor by factor.

Per solve (velocity_solve.py _solve_lines_hip, csrc/ns_condense.hip):
  two nested interior solves, each reading  Xi (element-interior inverses), Aei (edge <- interior),
                                            Yie (interior <- edge), Ed/El (forward) and Eu (back) edge
                                            block-Thomas factors, the right-hand side lines;
                                            the second also aIB and x_B -- by default (ABI 11) its element
                                            step reads Xi A_iB and A_ei Xi A_iB instead of Xi and Aei;
  the interface right-hand side            aBI, the interface lines, y_I;
  the interface sweep (block Thomas)       D0, F_L = [D_L^-1 | -D_L^-1 S_lo] (m x 2m) forward,
                                            Uh_L (m x m) back; or the CR operators.
Writes: the solution lines, the nested work arrays (T, C, Ye) and y_I.

Under rocprofv3 --kernel-trace, tools/trace_window.py <csv> SOLVES cond_fwd_kernel 2 splits the last
SOLVES solves per kernel; the bytes here divide by those durations.

python tools/vsolve_probe.py [--ne 128 --P 12 --Ra 1e6 --solves 20 --ab-edge 1 --ab-back 1]
  (--ab-edge: first the ABI-9 edge sweep; --ab-back: first the ABI-10 back substitution)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def nbytes(t):
    return 0 if t is None else t.numel() * t.element_size()


def account(vs, back=None):
    """Algorithmic bytes of one solve, by factor (back: the back-substitution path, vs.nested_back)."""
    XiT, AeiT, YieT, SeT = vs._hipT
    back = back or vs.nested_back
    b = {}
    if back == "coupled" and getattr(vs, "_hipB", None) is not None:   # ABI 11
        XiBT, AXBT, ABYT = vs._hipB
        b["Xi (element-interior inverses)"] = nbytes(XiT)
        b["Aei"] = nbytes(AeiT)
        b["ABY (interface right-hand side)"] = nbytes(ABYT)
        b["XiB + AXB (back substitution)"] = nbytes(XiBT) + nbytes(AXBT)
        b["Yie (back substitution)"] = nbytes(YieT)
        # T written, read by the interface sums, read + written by the back step, read by the last step; C
        # written, read + written, read by the edge sweeps; the interface partial sums written and read once
        b["T, C, partial-sum work"] = 4 * nbytes(vs._work[0]) + 4 * nbytes(vs._work[1]) + 2 * nbytes(vs._work[5])
    else:
        b["Xi (element-interior inverses) x2"] = 2 * nbytes(XiT)
        b["Aei x2"] = 2 * nbytes(AeiT)
        b["Yie x2"] = 2 * nbytes(YieT)
    if vs._edge_thomas:
        Ed, El, Eu = vs._EtT
        b["edge Thomas Ed+El+Eu x2"] = 2 * (nbytes(Ed) + nbytes(El) + nbytes(Eu))
    else:
        b["edge Schur inverses x2"] = 2 * nbytes(SeT)
    b["aIB + aBI"] = nbytes(vs.aIB) + nbytes(vs.aBI)
    if getattr(vs, "_tw", None) is not None:   # two-ended sweep
        k, D0, E0, FT, FB, FM, UhT, UhB = vs._tw
        b["sweep FT_L + FB_L (m x 2m)"] = nbytes(FT) + nbytes(FB)
        b["sweep FM (m x 3m, middle line)"] = nbytes(FM)
        b["sweep UhT_L + UhB_L (m x m)"] = nbytes(UhT) + nbytes(UhB)
        b["sweep D0 + E0"] = nbytes(D0) + nbytes(E0)
    elif getattr(vs, "_th", None) is not None:
        D0, F, Uh = vs._th
        b["sweep F_L (m x 2m)"] = nbytes(F)
        b["sweep Uh_L (m x m)"] = nbytes(Uh)
        b["sweep D0"] = nbytes(D0)
    elif getattr(vs, "_cr", None):
        b["CR operators"] = sum(nbytes(l[1]) + nbytes(l[4]) for l in vs._cr) + nbytes(vs._cr_top[1])
    NX, m = vs.NX, vs.m
    vec = NX * m * 8
    # right-hand side lines read twice (both nested solves), solution written once, interface lines
    b["vectors (rhs x2, solution, interface)"] = 3 * vec + 4 * (vs.nex + 1) * m * 8
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ne", type=int, default=128)
    ap.add_argument("--P", type=int, default=12)
    ap.add_argument("--Ra", type=float, default=1e6)
    ap.add_argument("--solves", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--ab-edge", type=int, default=1, help="also time the ABI-9 runtime-width edge sweep")
    ap.add_argument("--ab-oneended", type=int, default=0,
                    help="also time the one-ended edge sweep (EDGE_THOMAS = 2) against the two-ended one (ABI 12)")
    ap.add_argument("--ab-back", type=int, default=1,
                    help="also time the ABI-10 back substitution (a second nested solve through Xi)")
    args = ap.parse_args()
    from sem_amd.solvers import NavierStokesSolver
    Re, Pr = 1e3, 0.71
    dev = torch.device("cuda", 0)
    ns = NavierStokesSolver(1.0, 1.0, Re, args.Ra / Pr, args.P, args.ne, args.ne, mtol=1e-10, mtol_newton=1e-10,
                            iprint=[])
    N = ns.N
    r = np.random.default_rng(5)
    # a non-trivial linearisation: smooth velocities of O(1e-2), conduction temperature
    x, y = ns.points
    u0 = 1e-2 * np.sin(np.pi * x) * np.sin(2 * np.pi * y)
    v0 = -1e-2 * np.sin(2 * np.pi * x) * np.sin(np.pi * y)
    ns._get_residuals(u0, v0, np.zeros(N), 0.5 - x)
    ns._calc_jacobians(u0, v0)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    vs = ns._velocity_solver()
    torch.cuda.synchronize(dev)
    out = {"config": f"velocity solve {args.ne}x{args.ne} P={args.P}", "N": N, "factor_s": time.perf_counter() - t0,
           "resident_GB": torch.cuda.memory_allocated(dev) / 1e9, "edge_thomas": bool(vs._edge_thomas),
           "sweep": vs.sweep, "sweep_form": vs.sweep_form, "graph": getattr(vs, "_graph", None) is not None}
    bu, bv = (ns._dev(r.uniform(-1, 1, N)) for _ in range(2))

    def timed():
        for _ in range(3):
            vs.solve(bu, bv)
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(args.solves):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            xu, xv = vs.solve(bu, bv)
            b.record()
            torch.cuda.synchronize(dev)
            ts.append(a.elapsed_time(b))
        return ts, xu, xv

    if args.ab_edge and vs._edge_thomas:   # A/B first, so the trace's last `solves` solves are the default's
        from sem_amd import _lib
        lib = _lib.load()
        _lib.check(lib.sem_set_tuning(_lib.TUNE_EDGE_THOMAS, 1))
        vs.capture()
        ts_rt, xu_rt, xv_rt = timed()
        _lib.check(lib.sem_set_tuning(_lib.TUNE_EDGE_THOMAS, 0))
        vs.capture()
        out["abi9_edge_sweep_solve_ms_median"] = float(np.median(ts_rt))
    one_ended = args.ab_oneended and getattr(vs, "_edge_twisted", False)
    out["edge_twisted"] = bool(getattr(vs, "_edge_twisted", False))
    if one_ended:
        from sem_amd import _lib
        lib = _lib.load()
        _lib.check(lib.sem_set_tuning(_lib.TUNE_EDGE_THOMAS, 2))
        vs.capture()
        ts_oe, xu_oe, xv_oe = timed()
        _lib.check(lib.sem_set_tuning(_lib.TUNE_EDGE_THOMAS, 0))
        vs.capture()
        out["one_ended_edge_solve_ms_median"] = float(np.median(ts_oe))
    if args.ab_back and getattr(vs, "_hipB", None) is not None:
        vs.nested_back = "full"
        vs.capture()
        ts_full, xu_f, xv_f = timed()
        vs.nested_back = "coupled"
        vs.capture()
        bf = sum(account(vs, "full").values())
        med_f = float(np.median(ts_full))
        out["full_back_solve_ms_median"] = med_f
        out["full_back_bytes_per_solve"] = bf
        out["full_back_frac_8TBs"] = bf / (med_f * 1e-3) / 8e12
    ts, xu, xv = timed()
    if args.ab_back and getattr(vs, "_hipB", None) is not None:
        out["coupled_vs_full_rel_diff"] = float(max((xu - xu_f).abs().max(), (xv - xv_f).abs().max())
                                                / max(xu.abs().max(), xv.abs().max()))
    if args.ab_edge and vs._edge_thomas:
        out["abi9_vs_templated_rel_diff"] = float(max((xu - xu_rt).abs().max(), (xv - xv_rt).abs().max())
                                                  / max(xu.abs().max(), xv.abs().max()))
    if one_ended:
        out["one_ended_vs_two_ended_rel_diff"] = float(max((xu - xu_oe).abs().max(), (xv - xv_oe).abs().max())
                                                       / max(xu.abs().max(), xv.abs().max()))
    ju, jv, _ = ns._get_dresiduals(xu, xv, torch.zeros_like(xu))
    out["rel_residual"] = float(max((ju - bu).abs().max(), (jv - bv).abs().max()) / max(bu.abs().max(), bv.abs().max()))
    acc = account(vs)
    tot = sum(acc.values())
    med = float(np.median(ts))
    out.update({"solve_ms_median": med, "solve_ms_min": float(min(ts)), "bytes_per_solve": tot,
                "bytes_by_factor": acc, "achieved_GBs": tot / (med * 1e-3) / 1e9,
                "frac_8TBs": tot / (med * 1e-3) / 8e12, "device": torch.cuda.get_device_name(dev)})
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
