"""Device direct solve of the Navier-Stokes velocity Jacobian.

Replaces the reference's host SuperLU of the 2N x 2N velocity Jacobian
(NavierStokes_Solver.py:176-192: `bmat` -> Dirichlet rows -> `splu`, then `lu.solve` twice per
Schur-complement matvec) with a static condensation that fits the structured SEM mesh:

* Node lines in the x-major numbering (SEM.py:110) are either *interface* lines x = L P
  (L = 0..N_ex) or one of the P-1 *interior* lines of an element column.  The operators couple a
  node only to nodes of the same line (y direction) and of the same element column (x direction),
  so the interior lines of column e couple to each other and to interface lines e and e+1 only.
* `sem_velocity_blocks` (HIP, sem_amd/csrc/ns_velocity.hip) writes the pieces: one dense block
  A_II per element column ((P-1) 2 N_y unknowns), the dense interface-line blocks D, and the
  diagonal line-to-line couplings.
* Factor: batched pivoted LU of the A_II blocks (rocSOLVER through torch), W = A_II^-1 A_IB, the
  interface Schur complement S = A_BB - A_BI W (block tridiagonal over the N_ex+1 interface lines,
  blocks of 2 N_y), and its block-LU (block Thomas) with explicit inverses of the pivot blocks.
* Solve: interior forward solve, the interface sweep (2 (N_ex+1) small GEMVs), interior back
  substitution.

Everything is device memory: cfg3 (32^2, P = 8) holds 3.3 GB of A_II factors, cfg4 (48^2, P = 8)
11 GB, well inside one MI355X's 288 GB.  The algebra runs on any torch device, so the
condensation itself is unit-tested on CPU against SciPy's sparse solve
(tests/test_velocity_solve.py); the block assembly needs the GPU.
"""
import torch


class VelocityJacobianSolver:
    """x = J^-1 b for the velocity Jacobian J of one linearisation, J given by its condensation pieces."""

    def __init__(self, P, nex, ney, device, interior="lu"):
        if P < 1 or nex < 1 or ney < 1:
            raise ValueError("bad mesh")
        if interior not in ("lu", "inverse"):
            raise ValueError("interior must be 'lu' or 'inverse'")
        self.P, self.nex, self.ney = P, nex, ney
        self.NY, self.NX = ney * P + 1, nex * P + 1
        self.m = 2 * self.NY
        self.nI = (P - 1) * self.m
        self.device = torch.device(device)
        self.interior = interior
        self.factored = False

    # ------------------------------------------------------------------ assembly
    def empty_blocks(self):
        """Zeroed storage for the pieces, in sem_velocity_blocks' layout."""
        P, nex, m, nI = self.P, self.nex, self.m, self.nI
        z = dict(dtype=torch.float64, device=self.device)
        return dict(AII=torch.zeros((nex, nI, nI), **z) if P > 1 else None,
                    D=torch.zeros((nex + 1, m, m), **z),
                    aIB=torch.zeros((nex, P - 1, 2, m), **z) if P > 1 else None,
                    aBI=torch.zeros((nex, 2, P - 1, m), **z) if P > 1 else None,
                    E=torch.zeros((nex, m), **z), F=torch.zeros((nex, m), **z))

    # ------------------------------------------------------------------ factorisation
    def factor(self, AII, D, aIB, aBI, E, F):
        """Condense and factor.  AII is consumed (its storage is reused for the LU factors)."""
        P, nex, m = self.P, self.nex, self.m
        if P > 1:
            LU, piv, info = torch.linalg.lu_factor_ex(AII)
            del AII
            if int(info.max().item()) > 0:
                raise RuntimeError("velocity Jacobian: singular interior block")
            # dense A_IB (nex, nI, 2m): rows (l, r), column block s holds aIB[e, l, s, r] on its diagonal
            AIB = torch.diag_embed(aIB).permute(0, 1, 3, 2, 4).reshape(nex, self.nI, 2 * m)
            W = torch.linalg.lu_solve(LU, piv, AIB)
            del AIB
            Wr = W.view(nex, P - 1, m, 2, m)
            # C[e, s, r, t, k] = sum_l aBI[e, s, l, r] W[e, l, r, t, k]: A_BI W for both interface lines
            C = torch.zeros((nex, 2, m, 2, m), dtype=torch.float64, device=self.device)
            for li in range(P - 1):
                C += aBI[:, :, li, :, None, None] * Wr[:, None, li]
            S_diag = D.clone()
            S_diag[:-1] -= C[:, 0, :, 0, :]
            S_diag[1:] -= C[:, 1, :, 1, :]
            S_up = torch.diag_embed(E) - C[:, 0, :, 1, :]
            S_lo = torch.diag_embed(F) - C[:, 1, :, 0, :]
            del C
            if self.interior == "inverse":
                eye = torch.eye(self.nI, dtype=torch.float64, device=self.device).expand(nex, -1, -1)
                self.Ainv = torch.linalg.lu_solve(LU, piv, eye)
                del LU, piv
                self.LU = self.piv = None
            else:
                self.LU, self.piv = LU, piv
            self.W = W.view(nex, self.nI, 2, m)
            self.aBI = aBI
        else:
            S_diag, S_up, S_lo = D, torch.diag_embed(E), torch.diag_embed(F)
        # block Thomas on the interface lines: Dt[0] = S_diag[0], Uh[L] = Dt[L]^-1 S_up[L],
        # Dt[L+1] = S_diag[L+1] - S_lo[L] Uh[L]; explicit (pivoted) inverses of the pivot blocks
        Dinv = torch.empty((nex + 1, m, m), dtype=torch.float64, device=self.device)
        Uh = torch.empty((nex, m, m), dtype=torch.float64, device=self.device)
        Dt = S_diag[0]
        for L in range(nex + 1):
            if L > 0:
                Dt = S_diag[L] - S_lo[L - 1] @ Uh[L - 1]
            Dinv[L] = torch.linalg.inv(Dt)
            if L < nex:
                Uh[L] = Dinv[L] @ S_up[L]
        self.Dinv, self.Uh, self.S_lo = Dinv, Uh, S_lo
        self.factored = True

    # ------------------------------------------------------------------ solve
    def solve(self, bu, bv):
        """(J^-1 [bu; bv]) split as (xu, xv); bu, bv are length-N vectors in the x-major numbering."""
        if not self.factored:
            raise RuntimeError("factor() first")
        P, nex, m, NX, NY = self.P, self.nex, self.m, self.NX, self.NY
        B = torch.stack((bu.reshape(NX, NY), bv.reshape(NX, NY)), dim=1).reshape(NX, m)
        g = B[0::P].clone()                                    # interface lines (nex+1, m)
        if P > 1:
            bI = B[:-1].reshape(nex, P, m)[:, 1:, :].reshape(nex, self.nI, 1)
            if self.interior == "inverse":
                yI = torch.bmm(self.Ainv, bI)
            else:
                yI = torch.linalg.lu_solve(self.LU, self.piv, bI)
            yIr = yI.view(nex, P - 1, m)
            g[:-1] -= (self.aBI[:, 0] * yIr).sum(1)
            g[1:] -= (self.aBI[:, 1] * yIr).sum(1)
        # interface sweep
        z = torch.empty_like(g)
        z[0] = self.Dinv[0] @ g[0]
        for L in range(1, nex + 1):
            z[L] = self.Dinv[L] @ (g[L] - self.S_lo[L - 1] @ z[L - 1])
        xB = z
        for L in range(nex - 1, -1, -1):
            xB[L] = z[L] - self.Uh[L] @ xB[L + 1]
        out = torch.empty((NX, m), dtype=torch.float64, device=self.device)
        out[0::P] = xB
        if P > 1:
            xI = yI.view(nex, self.nI) - (torch.bmm(self.W[:, :, 0, :], xB[:-1, :, None])
                                          + torch.bmm(self.W[:, :, 1, :], xB[1:, :, None]))[..., 0]
            out[:-1].view(nex, P, m)[:, 1:, :] = xI.view(nex, P - 1, m)
        out = out.view(NX, 2, NY)
        return out[:, 0, :].reshape(-1), out[:, 1, :].reshape(-1)
