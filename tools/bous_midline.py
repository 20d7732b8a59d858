"""Benchmark check of a Boussinesq state (tools/bous_solve.py checkpoint, [T, u, v, p] on an N_e^2, P
mesh): u_max * Re * Pr on the vertical midline x = 0.5 and v_max * Re * Pr on the horizontal midline
y = 0.5, the quantities of de Vahl Davis (1983), evaluated on the host with the oracle's spectral
interpolation (SEM.py:248-273 restated).  Test/analysis infrastructure: reads a saved state, no GPU.

python tools/bous_midline.py STATE.npy --ne 48 --P 8 [--Re 1e3 --Pr 0.71]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("state")
    ap.add_argument("--ne", type=int, default=48)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--Re", type=float, default=1e3)
    ap.add_argument("--Pr", type=float, default=0.71)
    args = ap.parse_args()
    from oracle import sem_oracle as O
    P, ne = args.P, args.ne
    N = (ne * P + 1) ** 2
    x = np.load(args.state)
    u, v = x[N:2 * N], x[2 * N:3 * N]
    pe = O.element_nodes(P, ne, ne, 1.0 / ne, 1.0 / ne)
    s = np.linspace(0.0, 1.0, 2001)
    k = args.Re * args.Pr
    um = O.eval_interpolation(O.scatter(u, P, ne, ne), pe, np.meshgrid([0.5], s, indexing="ij"))[0] * k
    vm = O.eval_interpolation(O.scatter(v, P, ne, ne), pe, np.meshgrid(s, [0.5], indexing="ij"))[:, 0] * k
    i, j = int(um.argmax()), int(vm.argmax())
    print(json.dumps({"state": os.path.basename(args.state), "mesh": f"{ne}x{ne} P={P}",
                      "u_max_midline": float(um[i]), "u_max_y": float(s[i]),
                      "v_max_midline": float(vm[j]), "v_max_x": float(s[j])}))


if __name__ == "__main__":
    main()
