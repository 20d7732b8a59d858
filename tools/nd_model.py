"""Byte model of one NS velocity solve: the line condensation the device runs now against a
nested-dissection (ND) factorisation of the same Jacobian with element-block separators in both directions -- the
analogue of the reference's `splu`, which orders by COLAMD (NavierStokes_Solver.py:184).

Current scheme (sem_amd/solvers/velocity_solve.py): every element's interior is condensed (leaf step), every element
column's edges are condensed per column (edge step), and the interface system -- block tridiagonal over the N_ex + 1
interface lines, DENSE m x m blocks (m = ncomp N_y: the column interiors couple every node of a line to every
other) -- is swept by block Thomas: per line the forward operator F_L (m x 2m) and the back operator Uh_L (m x m).

ND: recursive bisection of the element grid along its longer side at the middle element edge.  A separator is the
skeleton nodes (element-edge nodes) of that edge line inside the piece; its front is the separator plus the piece's
perimeter nodes that belong to ancestor separators (Dirichlet boundary rows are identity rows and decouple).  A
front's LU holds |S|^2 + 2 |S| |B| entries (the separator block and the L / U panels to the boundary), and a solve
reads L in the forward pass and U in the back pass -- every entry once.  Leaves are single elements whose interiors
are condensed exactly as now (Xi, A_ie, A_ei), so the leaf bytes are the current scheme's element-interior bytes.

    python tools/nd_model.py            # cfg4 and cfg5 (and cfg3), table to stdout
Validation: the current scheme's model against the measured per-solve reads of the cfg5 kernel trace
(profiles/r04/cfg5_vsolve/final_trace/: sweep GEMVs 28.9 GB, element steps 9.07 + 1.72 + 1.43 GB).
"""
import argparse
import json


def current_scheme(P, nex, ney, nc=2):
    NY = ney * P + 1
    m = nc * NY
    ne1 = nc * (P - 1)                      # unknowns of an element edge (without its end vertices)
    ni = ne1 * (P - 1)                      # unknowns of an element interior
    E = nex * ney
    # element steps (ABI 11): forward reads Xi (ni^2) and A_ei (2 ne1 x ni) per element, the coupled back step reads
    # Xi A_iB (ni x 2 ne1) and A_ei Xi A_iB (2 ne1 x 2 ne1), the back step Yie (ni x 2 ne1); edge sweeps ~(ney+1) ne1^2 x 3
    elem = E * (ni * ni + 2 * ne1 * ni) * 8
    coupled = E * (ni * 2 * ne1 + 4 * ne1 * ne1) * 8
    back = E * (ni * 2 * ne1) * 8
    edges = 2 * nex * (ney + 1) * 3 * ne1 * ne1 * 8
    sweep = (nex + 1) * 3 * m * m * 8       # F_L (m x 2m) + Uh_L (m x m) per interface line
    resident = (nex + 1) * 3 * m * m * 8 + E * (ni * ni + 4 * ne1 * ni + 8 * ne1 * ne1) * 8
    return {"element_steps_GB": (elem + coupled + back) / 1e9, "edge_sweeps_GB": edges / 1e9,
            "interface_sweep_GB": sweep / 1e9, "total_GB": (elem + coupled + back + edges + sweep) / 1e9,
            "factor_resident_GB": resident / 1e9, "dependent_launches": (nex + 1) + 2 * 3 + 2}


def nd_scheme(P, nex, ney, nc=2, leaf_GB=None):
    """Skeleton ND on the element grid; separators along element edges; nodes counted with ncomp unknowns."""
    fronts = []

    def perim_nodes(x0, x1, y0, y1):
        """Skeleton nodes on the piece's perimeter that are not on the domain boundary (ancestor separators)."""
        n = 0
        if x0 > 0:
            n += (y1 - y0) * P + 1
        if x1 < nex:
            n += (y1 - y0) * P + 1
        if y0 > 0:
            n += (x1 - x0) * P + 1
        if y1 < ney:
            n += (x1 - x0) * P + 1
        return n

    def rec(x0, x1, y0, y1, level):
        a, b = x1 - x0, y1 - y0
        if a == 1 and b == 1:
            return
        if a >= b:                      # vertical separator at the middle element edge x = xm
            xm = (x0 + x1) // 2
            s = b * P - 1               # nodes strictly inside the piece on that line
            rec(x0, xm, y0, y1, level + 1)
            rec(xm, x1, y0, y1, level + 1)
        else:
            ym = (y0 + y1) // 2
            s = a * P - 1
            rec(x0, x1, y0, ym, level + 1)
            rec(x0, x1, ym, y1, level + 1)
        fronts.append((level, nc * s, nc * perim_nodes(x0, x1, y0, y1)))

    rec(0, nex, 0, ney, 0)
    entries = sum(S * S + 2 * S * B for _, S, B in fronts)
    levels = max(l for l, _, _ in fronts) + 1
    per_level = {}
    for l, S, B in fronts:
        per_level[l] = per_level.get(l, 0) + (S * S + 2 * S * B) * 8
    top = max(S for _, S, _ in fronts)
    flops = sum((2 / 3) * S ** 3 + 2 * S * S * B + 2 * S * B * B for _, S, B in fronts)
    return {"separator_factors_GB": entries * 8 / 1e9, "leaf_element_GB": leaf_GB,
            "total_GB": entries * 8 / 1e9 + (leaf_GB or 0.0), "fronts": len(fronts), "levels": levels,
            "largest_front": top, "factor_TFLOP": flops / 1e12,
            "GB_by_level": {str(k): round(v / 1e9, 3) for k, v in sorted(per_level.items())},
            "dependent_launches": 2 * levels}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    for name, P, ne in (("cfg3", 8, 32), ("cfg4", 8, 48), ("cfg5", 12, 128)):
        cur = current_scheme(P, ne, ne)
        nd = nd_scheme(P, ne, ne, leaf_GB=cur["element_steps_GB"] + cur["edge_sweeps_GB"])
        rec = {"config": name, "P": P, "ne": ne, "current": cur, "nested_dissection": nd,
               "bytes_ratio_current_over_nd": cur["total_GB"] / nd["total_GB"],
               "interface_ratio": cur["interface_sweep_GB"] / nd["separator_factors_GB"]}
        rows.append(rec)
        print(json.dumps(rec))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
