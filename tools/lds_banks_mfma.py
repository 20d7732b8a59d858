"""LDS bank-conflict model of apply_tp_mfma's accesses (sem_amd/csrc/sem_ops.hip), per tile config and layout.

Model (MI355X_MICROARCH.md, LDS): ds_read_b64 in two 32-lane groups, bank = dword mod 64; ds_write_b64 in four
16-lane groups, bank = dword mod 32; each extra distinct dword on a busy bank costs one cycle.  Every access of
one workgroup (staging writes, phase A / B operand reads, result writes, epilogue reads) is enumerated with the
kernel's lane mapping; the script prints the LDS cycles and the conflict cycles per access, for the Ts pitch and
the swizzle given.

python tools/lds_banks_mfma.py [P TX TY NW]
"""
import collections
import sys

R64 = [range(0, 32), range(32, 64)]
W64 = [range(i, i + 16) for i in range(0, 64, 16)]


def cycles(addrs, groups, nbanks):
    """addrs: {lane: double index}; returns (cycles, ideal cycles)."""
    tot = ideal = 0
    for g in groups:
        banks = collections.defaultdict(set)
        for lane in g:
            if lane in addrs:
                a = 2 * addrs[lane]
                for d in (a, a + 1):
                    banks[d % nbanks].add(d)
        if banks:
            tot += max(len(s) for s in banks.values())
            ideal += 1
    return tot, ideal


def pitch18(w):
    return w + ((18 - (w % 32)) + 32) % 32


def model(P, TX, TY, NW, PT=None, swz=lambda r, c: c, FLP=0, label="", SW=0):
    n = P + 1
    BX, BY = TX * P, TY * P
    NLB, NCB = (BX + 15) // 16, (BY + 15) // 16
    KS = (n + 3) // 4
    RX = max(TX * P + 4 * KS, P + 16 * NLB)
    RY = max(TY * P + 4 * KS, P + 16 * NCB)
    PT = PT or pitch18(RY)
    EC, FL = 16 * NCB, 16 * NLB
    FLN = FL * n + FLP      # FK pitch per element row (FLP: padding)
    THREADS = 64 * NW
    ts = lambda r, c: r * PT + swz(r, c)  # noqa: E731
    acc = collections.defaultdict(lambda: [0, 0])

    def add(name, addrs, groups, nb):
        c, i = cycles(addrs, groups, nb)
        acc[name][0] += c
        acc[name][1] += i

    # staging writes: idx = tid + s THREADS, (rr, cc) = divmod(idx, SW or RY); SW > RY: rows padded to SW slots
    SWd = SW or RY
    NST = (RX * SWd + THREADS - 1) // THREADS
    for s in range(NST):
        for w in range(NW):
            ad = {}
            for l in range(64):
                idx = w * 64 + l + s * THREADS
                rr, cc = divmod(idx, SWd)
                if rr < RX and cc < RY:
                    ad[l] = ts(rr, cc)
            add("stage write", ad, W64, 32)
    # phase A reads: tasks (e, cb), lanes (lk, lr): Ts[(e P + 4 s + lk), P + cb 16 + lr]
    TA = (TX + 1) * NCB
    for task in range(TA):
        e, cb = divmod(task, NCB)
        for s in range(KS):
            ad = {l: ts(e * P + 4 * s + (l >> 4), P + cb * 16 + (l & 15)) for l in range(64)}
            add("phase A read", ad, R64, 64)
    TB = (TY + 1) * NLB
    for task in range(TB):
        e, lbk = divmod(task, NLB)
        for s in range(KS):
            ad = {l: ts(P + lbk * 16 + (l & 15), e * P + 4 * s + (l >> 4)) for l in range(64)}
            add("phase B read", ad, R64, 64)
    # result writes: EK[(e n + i) EC + cb 16 + lr], i = lk + 4 r;  FK[(e FLN + line) n + lr]?  (line-major)
    for task in range(TA):
        e, cb = divmod(task, NCB)
        for r in range(4):
            ad = {l: (e * n + (l >> 4) + 4 * r) * EC + cb * 16 + (l & 15) for l in range(64) if (l >> 4) + 4 * r <= P}
            add("EK write", ad, W64, 32)
    for task in range(TB):
        e, lbk = divmod(task, NLB)
        for r in range(4):
            ad = {l: e * FLN + (lbk * 16 + (l >> 4) + 4 * r) * n + (l & 15) for l in range(64) if (l & 15) <= P}
            add("FK write", ad, W64, 32)
    # epilogue reads, per wave: idx = tid + q THREADS, (rl, c) = divmod(idx, BY)
    NMAIN = (BX * BY + THREADS - 1) // THREADS
    for q in range(NMAIN):
        for w in range(NW):
            lanes = {}
            for l in range(64):
                idx = w * 64 + l + q * THREADS
                if idx < BX * BY:
                    lanes[l] = divmod(idx, BY)
            add("epi Ts read", {l: ts(P + rl, P + c) for l, (rl, c) in lanes.items()}, R64, 64)
            add("epi EK read", {l: ((rl // P + 1) * n + rl % P) * EC + c for l, (rl, c) in lanes.items()}, R64, 64)
            add("epi EK(P) read", {l: ((rl // P) * n + P) * EC + c for l, (rl, c) in lanes.items()}, R64, 64)
            add("epi FK read", {l: (c // P + 1) * FLN + rl * n + c % P for l, (rl, c) in lanes.items()}, R64, 64)
            add("epi FK(P) read", {l: (c // P) * FLN + rl * n + P for l, (rl, c) in lanes.items()}, R64, 64)
    tc = sum(v[0] for v in acc.values())
    ti = sum(v[1] for v in acc.values())
    print(f"{label}: PT={PT} FK pitch {FLN}: {tc} LDS cycles per workgroup, {tc - ti} conflict cycles "
          f"({(tc - ti) / max(ti, 1):.2f} per instruction-group)")
    for k, (c, i) in acc.items():
        if c > i:
            print(f"    {k:16s} {c:6d} cycles, {c - i:5d} conflict")
    return tc - ti


def main():
    a = [int(x) for x in sys.argv[1:]] or [8, 2, 2, 4]
    P, TX, TY, NW = a
    model(P, TX, TY, NW, label="current (pitch18, no swizzle)")
    best = None
    for PT in range(32, 80):
        for sw in range(4):
            def swz(r, c, sw=sw):
                if sw == 0:
                    return c
                if sw == 1:
                    return c ^ (2 * ((r >> 1) & 7))
                if sw == 2:
                    return c ^ (2 * (r & 7))
                return c ^ (((r >> 1) & 3) << 2)
            if max(swz(r, c) for r in range(64) for c in range(48)) >= PT:
                continue
            import io
            import contextlib
            with contextlib.redirect_stdout(io.StringIO()):
                cc = model(P, TX, TY, NW, PT=PT, swz=swz, FLP=8)
            if best is None or cc < best[0]:
                best = (cc, PT, sw)
    print("best search:", best)
    if best:
        sw = best[2]
        for SW in (0, 32):
            model(P, TX, TY, NW, PT=best[1], swz=lambda r, c: [c, c ^ (2 * ((r >> 1) & 7)), c ^ (2 * (r & 7)),
                                                                c ^ (((r >> 1) & 3) << 2)][sw], FLP=8,
                  label=f"best, staging rows of {SW or 'RY'} slots", SW=SW)


if __name__ == "__main__":
    main()
