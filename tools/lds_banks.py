"""LDS bank-conflict count of the NS band kernel's Y-phase accesses (sem_amd/csrc/ns_apply.hip), per order P.

Model (MI355X_MICROARCH.md, LDS): ds_read_b64 is serviced in two 32-lane groups, bank = dword mod 64;
ds_write_b64 in four 16-lane groups, bank = dword mod 32; an extra distinct dword on a busy bank costs one
cycle.  For each P it counts the cycles of the staged-window reads ((P + r) PIT + b P + q, q = 0..2P) and the
Y-sum stores (r YP + b P + j) for the two lane mappings (lane -> (line r, element b), element fastest
or line fastest) and the two Y-sum pitches (BY, PIT).  NsBand<P>::RF picks the line-fastest mapping where
it wins.    python tools/lds_banks.py
"""
import collections

R64 = [range(0, 32), range(32, 64)]
W64 = [range(i, i + 16) for i in range(0, 64, 16)]


def cycles(addrs, groups, nbanks):
    tot = 0
    for g in groups:
        banks = collections.defaultdict(set)
        for lane in g:
            if lane in addrs:
                a = 2 * addrs[lane]
                for d in (a, a + 1):
                    banks[d % nbanks].add(d)
        tot += max((len(s) for s in banks.values()), default=0)
    return tot


def main():
    print("P  mapping        window-reads (ideal)   Y-sum stores pitch BY / PIT (ideal)")
    for P in range(1, 17):
        TYE = max(1, 64 // P)
        BY = TYE * P
        PIT = (BY + P + 1) | 1
        for rf in (False, True):
            def rb(lane):
                return (lane % P, lane // P) if rf else (lane // TYE, lane % TYE)
            lanes = range(P * TYE)
            rd = sum(cycles({l: (P + rb(l)[0]) * PIT + rb(l)[1] * P + q for l in lanes}, R64, 64)
                     for q in range(2 * P + 1))
            st = [sum(cycles({l: rb(l)[0] * yp + rb(l)[1] * P + j for l in lanes}, W64, 32) for j in range(P))
                  for yp in (BY, PIT)]
            print(f"{P:2d} {'line-fastest' if rf else 'elem-fastest'}  {rd:5d} ({2 * (2 * P + 1):4d})"
                  f"            {st[0]:5d} / {st[1]:5d} ({4 * P:4d})")


if __name__ == "__main__":
    main()
