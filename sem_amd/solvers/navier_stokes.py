"""Navier-Stokes solver counterpart on the device operators.

Mirrors Solvers/NavierStokes_Solver.py:10-306 (same constructor, same private
methods the OpenMDAO component calls, same errors).  The operator applies run on
the GPU as fused launches:

  * `_get_residuals`  (:93-121): res_u = Sys u + G_x p, res_v = Sys v + G_y p - Gr/Re M T,
    res_cont = G_x u + G_y v, with the reference's Dirichlet / pinned-pressure /
    artificial-Neumann (`K[mask,:] @ p`) rows -- one sem_ns_apply launch for all three outputs.
  * `_calc_jacobians` (:123-136): Re diag(G_x u) ... as closed-form operators.
  * `_get_dresiduals` (:138-160): the velocity Jacobian blocks applied matrix-free, one launch.

`_get_update` keeps the reference's algorithm -- a direct velocity solve inside a pressure
Schur-complement Krylov solve with the mass-diagonal preconditioner (NavierStokes_Solver.py:162-236)
-- entirely on the device: the velocity Jacobian is factored by static condensation over node
lines (sem_amd/solvers/velocity_solve.py, blocks written by the sem_velocity_blocks HIP kernel)
instead of host SuperLU, and the Schur system runs the device GMRES.  No CSR matrix is formed.
"""
import gc
import os
import time

import numpy as np
import torch

from .. import SEM, _lib
from ..device import get_mesh, no_gc
from ..krylov import Recycle, gcro, gmres
from ..operators import ConvectionTensor, SEMOperator
from ..tracing import phase
from .convection_diffusion import DirichletRows
from .nested_dissection import NestedDissectionSolver
from .velocity_solve import VelocityJacobianSolver


def _mass_diagonal(P, nex, ney, dx, dy):
    """Diagonal of the assembled mass matrix (SEM.py:170-183): (dx/2)(dy/2) wx_g wy_g with the GLL
    weights summed over the elements holding each 1-D node."""
    from .. import GLL
    w = GLL.standard_nodes(P)[1]
    wx, wy = np.zeros(nex * P + 1), np.zeros(ney * P + 1)
    for e in range(nex):
        wx[e * P:e * P + P + 1] += w
    for e in range(ney):
        wy[e * P:e * P + P + 1] += w
    return ((dx / 2) * (dy / 2)) * np.outer(wx, wy).ravel()


_ALL_SIDES = _lib.SIDE_W | _lib.SIDE_E | _lib.SIDE_S | _lib.SIDE_N


class NavierStokesSolver:
    def __init__(self, L_x: float, L_y: float, Re: float, Gr: float, P: int, N_ex: int, N_ey: int,
                 v_W: float = 0, v_E: float = 0, u_S: float = 0, u_N: float = 0,
                 mtol=1e-7, mtol_newton=1e-5, iprint: list = ['NEWTON_suc', 'NEWTON_iter'],  # noqa: B006
                 max_basis: int = 3000, velocity_interior: str = "auto", velocity_graph: bool = True,
                 recycle_bytes: float = 0.0, velocity_sweep: str = "auto", schur_precond: str = "mass",
                 partition=None, partition_update: str = "distributed"):
        """partition: a sem_amd.parallel.Partition -- the solver then holds one element-column strip per
        rank: _get_residuals / _calc_jacobians / _get_dresiduals run the fused strip launch and sum the
        interface lines of all three outputs with one collective.  partition_update: "distributed"
        (default) -- _get_update runs on the strips: the velocity Jacobian is factored by the
        element-partitioned condensation (strip_solve.StripLineSolver: each rank its own columns, a
        reduced system over the strip-boundary lines shared by all), and the Schur-complement Krylov
        solve runs over the strips (inner products all-reduced); "central" -- rank 0's whole-mesh
        counterpart (_central_solver) solves and the update is broadcast.  The reference methods take
        and return global NumPy vectors (local strips when given device tensors).
        recycle_bytes: device memory for a recycled Krylov subspace of the Schur-complement solves
        (sem_amd.krylov.Recycle, GCRO; 0 = off, the default): consecutive _get_update calls with one
        linearisation -- the Boussinesq coupler's block-Jacobi preconditioner -- then start from the
        earlier solves' spaces.  Measured (tools/recycle_probe.py, profiles/r02/bous): 5-8x fewer Schur
        matvecs on consistent right-hand sides, but the Arnoldi-relation error of the recycled space
        puts a floor near 1e-8 relative under the residual, above the couplers' mtol_internal = 1e-13,
        so inside the coupler it stagnates; off by default.
        velocity_interior: the velocity-Jacobian factorisation -- "auto" (default): nested dissection of the element
        grid (solvers/nested_dissection.py; on a partitioned solver each strip's own dissection, StripNDSolver) when
        the Dirichlet rows are the whole perimeter (the reference's velocity mask) and P >= 2, else the line
        condensation; "nd": nested dissection; "nested" / "lu" / "inverse": the line condensation
        (solvers/velocity_solve.py, strip_solve.StripLineSolver) with its interior variants.
        schur_precond: right preconditioner of the Schur-complement Krylov solve.  "mass" (default):
        the reference's mass diagonal (NavierStokes_Solver.py:207-212); "pcd": a
        pressure-convection-diffusion approximation S^-1 ~ A_p^-1 F_p M^-1 on the continuity rows,
        A_p^-1 on the pressure rows the reference replaces (boundary K rows, pinned node), where
        A_p = K with the pinned row (factored once per solver by the one-component line
        condensation) and F_p = Sys of the linearisation.  Right preconditioning keeps the stopping
        test on the true Schur residual, so the reference's rule is unchanged; only the Krylov count
        falls (tools/pcd_probe.py).  It is opt-in because on the smallest meshes (4^2, P=4) the
        equal-order Jacobian is singular or nearly so, and which member of the near-null family of
        solutions a Krylov method returns depends on its preconditioner: the reference's golden
        velocities there are reproduced only by the reference's own preconditioner."""
        if schur_precond not in ("mass", "pcd"):
            raise ValueError("schur_precond must be 'mass' or 'pcd'")
        if velocity_interior not in ("auto", "nd", "nested", "lu", "inverse"):
            raise ValueError("velocity_interior must be 'auto', 'nd', 'nested', 'lu' or 'inverse'")
        if partition_update not in ("distributed", "central"):
            raise ValueError("partition_update must be 'distributed' or 'central'")
        if partition is not None and schur_precond != "mass" and partition_update == "distributed":
            raise ValueError("the distributed update uses the mass-diagonal Schur preconditioner")
        self._partition_update = partition_update
        self._schur_precond, self._Ap = schur_precond, None
        self._iprint = iprint
        self._recycle_bytes, self._schur_recycle = recycle_bytes, None
        self._velocity_interior, self._velocity_graph = velocity_interior, velocity_graph
        self._velocity_sweep = velocity_sweep
        self._max_basis = max_basis
        self._velo = None
        self._Re, self._Gr = Re, Gr
        if self._Re == 0 and self._Gr != 0:
            raise ValueError('Cannot have Re == 0 and Gr != 0')
        self._Gr_over_Re = self._Gr / self._Re if self._Re != 0 else 0.
        self._mtol, self._mtol_newton = mtol, mtol_newton
        self._L_x, self._L_y = L_x, L_y
        self._P, self._N_ex, self._N_ey = P, N_ex, N_ey
        dx, dy = L_x / N_ex, L_y / N_ey
        self.points = SEM.global_nodes(P, N_ex, N_ey, L_x / N_ex, L_y / N_ey)
        self.points_e = SEM.element_nodes(P, N_ex, N_ey, dx, dy)
        self.N = (N_ex * P + 1) * (N_ey * P + 1)
        self._args = dict(L_x=L_x, L_y=L_y, Re=Re, Gr=Gr, P=P, N_ex=N_ex, N_ey=N_ey, v_W=v_W, v_E=v_E, u_S=u_S,
                          u_N=u_N, mtol=mtol, mtol_newton=mtol_newton, iprint=iprint, max_basis=max_basis,
                          velocity_interior=velocity_interior, velocity_graph=velocity_graph,
                          recycle_bytes=recycle_bytes, velocity_sweep=velocity_sweep, schur_precond=schur_precond)
        self._part, self._twin, self._lin, self._lin_sys = partition, None, None, None
        if partition is None:
            self._mesh = m = get_mesh(P, N_ex, N_ey, dx, dy)
            self._M = SEM.global_mass_matrix(P, N_ex, N_ey, dx, dy)
            self._K = SEM.global_stiffness_matrix(P, N_ex, N_ey, dx, dy)
            self._C_x, self._C_y = SEM.global_convection_matrices(P, N_ex, N_ey, dx, dy)
        else:   # matrix-free operators on this rank's strip
            self._mesh = m = partition.setup(P, N_ex, N_ey, dx, dy)
            self._M, self._K = SEMOperator(m, cM=1.0), SEMOperator(m, cK=1.0)
            self._C_x, self._C_y = ConvectionTensor(m, "x"), ConvectionTensor(m, "y")
        self._Sys = None
        self._Jac_u_u = self._Jac_u_v = self._Jac_v_u = self._Jac_v_v = None
        self._jac_kw, self._schur = None, None

        # Dirichlet values and masks, exactly as NavierStokes_Solver.py:78-94 builds them
        x, y = self.points
        du, dv, dpp = np.full(self.N, np.nan), np.full(self.N, np.nan), np.full(self.N, np.nan)
        dv[np.isclose(x, 0)] = v_W
        du[np.isclose(x, 0)] = 0
        dv[np.isclose(x, self._L_x)] = v_E
        du[np.isclose(x, self._L_x)] = 0
        du[np.isclose(y, 0)] = u_S
        dv[np.isclose(y, 0)] = 0
        du[np.isclose(y, self._L_y)] = u_N
        dv[np.isclose(y, self._L_y)] = 0
        dpp[int(self.N / 2)] = 0
        self._dirichlet_u, self._dirichlet_v, self._dirichlet_p = du, dv, dpp
        self._mask_bound = ~np.isnan(du)
        self._mask_dir_p = ~np.isnan(dpp)
        all_sides = _lib.SIDE_W | _lib.SIDE_E | _lib.SIDE_S | _lib.SIDE_N
        self._dir = DirichletRows(m, self._mask_bound, all_sides)
        self._dval_u = self._dev(np.where(self._mask_bound, du, 0.0))
        self._dval_v = self._dev(np.where(self._mask_bound, dv, 0.0))
        pins = np.nonzero(self._mask_dir_p)[0]
        if len(pins) > 1:
            raise ValueError("one pinned pressure node is supported")
        self._pin = int(pins[0]) if len(pins) else -1
        self._pin_val = float(dpp[self._pin]) if len(pins) else 0.0
        if partition is not None:
            # the reference's mass diagonal (NavierStokes_Solver.py:207-212) is the assembled one: on a
            # shared line both strips hold the whole-mesh value
            self._Mdiag = m.to_device(partition.local(_mass_diagonal(P, N_ex, N_ey, dx, dy)))
            self._pin_local = self._pin - m.dof_begin if 0 <= self._pin - m.dof_begin < m.n_local else -1
            return
        self._Mdiag = m.to_device(self._M.diagonal())
        # PCD row weights: 1/M on the continuity rows, 0 on the replaced rows (and the reverse)
        repl = self._mask_bound.copy()
        if self._pin >= 0:
            repl[self._pin] = True
        self._pcd_w = m.to_device(np.where(repl, 0.0, 1.0 / self._M.diagonal()))
        self._pcd_b = m.to_device(repl.astype(np.float64))

    # ------------------------------------------------------------------ helpers
    def _dev(self, a):
        """Device vector of this solver's (local) DOFs; a global NumPy vector is sliced to the strip."""
        if a is None:
            return None
        if self._part is not None and not isinstance(a, torch.Tensor):
            a = self._part.local(np.asarray(a))
        return self._mesh.to_device(a)

    def _out(self, t, like):
        if isinstance(like, torch.Tensor):
            return t
        if self._part is not None:
            t = self._part.gather(t)
        return t.cpu().numpy()

    def _global(self, a):
        """Global NumPy vector from a global NumPy vector or this rank's strip tensor."""
        if isinstance(a, torch.Tensor) and self._part is not None:
            return self._part.gather(a).cpu().numpy()
        return np.asarray(a.cpu() if isinstance(a, torch.Tensor) else a, dtype=np.float64)

    def _norm(self, *ys):
        if self._part is not None:
            return self._part.norm(*ys)
        return torch.sqrt(sum(y.square().sum() for y in ys)).item()

    def _amax(self, *ys):
        if self._part is not None:
            return self._part.amax(*ys)
        return max(y.abs().max().item() for y in ys)

    def _grad(self, x, which):
        """G_x x or G_y x, assembled across strips on a partitioned solver."""
        if self._part is None:
            return self._mesh.apply(x, **{which: 1.0})
        return self._part.step(x, **{which: 1.0})

    def _sys_kw(self, Sys):
        cX, cu, cY, cv, d = Sys._coeffs()
        return dict(c_stiff=Sys.cK, c_mass=Sys.cM, c_gradx=cX, cu=cu, c_grady=cY, cv=cv)

    def _ns_kw(self, pin_first):
        """Row replacements of sem_ns_apply: Dirichlet rows (mask_bound) and the pinned-pressure row."""
        return dict(pin=self._pin, pin_val=0.0 if not pin_first else self._pin_val, pin_first=pin_first,
                    **self._dir.kw())

    # ------------------------------------------------------------------ reference methods
    def _get_residuals(self, u, v, p, T):
        """NavierStokes_Solver.py:93-121: one fused launch (sem_ns_apply) for res_u, res_v, res_cont."""
        m = self._mesh
        U, V, Pp, Tt = self._dev(u), self._dev(v), self._dev(p), self._dev(T)
        Conv = self._Re * (SEM.tensordot(self._C_x, U, (1, 0)) + SEM.tensordot(self._C_y, V, (1, 0)))
        self._Sys = self._K + Conv
        if self._schur_recycle is not None:   # the Schur operator depends on Sys
            self._schur_recycle.reset()
        ru, rv, rc = (torch.empty_like(U) for _ in range(3))
        m.ns_apply(U, V, Pp, ru, rv, rc, **self._sys_kw(self._Sys), c_T=-self._Gr_over_Re, T=Tt,
                   dval_u=self._dval_u, dval_v=self._dval_v, **self._ns_kw(pin_first=True))
        if self._part is not None:
            self._part.assemble(ru, rv, rc)
            self._lin_sys = (U, V)   # Sys's velocity: part of the next linearisation
        return self._out(ru, u), self._out(rv, u), self._out(rc, u)

    def _calc_jacobians(self, u, v):
        """NavierStokes_Solver.py:123-136.  The Jacobians keep the Sys of this linearisation, as the
        reference's J_uu = Sys + ... does, even if _get_residuals runs again before they are used."""
        U, V = self._dev(u), self._dev(v)
        Re = self._Re
        if self._part is None:
            self._Jac_u_u = self._Sys + Re * SEM.tensordot(self._C_x, U, (2, 0))
            self._Jac_v_v = self._Sys + Re * SEM.tensordot(self._C_y, V, (2, 0))
            self._Jac_u_v = Re * SEM.tensordot(self._C_y, U, (2, 0))
            self._Jac_v_u = Re * SEM.tensordot(self._C_x, V, (2, 0))
        else:   # G u on a strip needs the interface exchange before it becomes a diagonal
            m = self._mesh
            self._Jac_u_u = self._Sys + SEMOperator(m, dg=[(Re, self._grad(U, "c_gradx"))])
            self._Jac_v_v = self._Sys + SEMOperator(m, dg=[(Re, self._grad(V, "c_grady"))])
            self._Jac_u_v = SEMOperator(m, dg=[(Re, self._grad(U, "c_grady"))])
            self._Jac_v_u = SEMOperator(m, dg=[(Re, self._grad(V, "c_gradx"))])
            self._lin = {"sys": self._lin_sys, "jac": (U, V), "stale": True}
        self._jac_kw = dict(self._sys_kw(self._Sys), juu=self._Jac_u_u._coeffs()[4], jvv=self._Jac_v_v._coeffs()[4],
                            juv=self._Jac_u_v._coeffs()[4], jvu=self._Jac_v_u._coeffs()[4])
        self._velo = None  # factorised on first use, reused until the next linearisation
        self._schur = None
        if self._schur_recycle is not None:
            self._schur_recycle.reset()

    def _get_dresiduals(self, du, dv, dp, dT=None):
        """NavierStokes_Solver.py:138-160: one fused launch (sem_ns_apply) for the three differentials."""
        m = self._mesh
        DU, DV, DP = self._dev(du), self._dev(dv), self._dev(dp)
        ru, rv, rc = (torch.empty_like(DU) for _ in range(3))
        m.ns_apply(DU, DV, DP, ru, rv, rc, **self._jac_kw, c_T=-self._Gr_over_Re if dT is not None else 0.0,
                   T=self._dev(dT), **self._ns_kw(pin_first=False))
        if self._part is not None:
            self._part.assemble(ru, rv, rc)
        return self._out(ru, du), self._out(rv, du), self._out(rc, du)

    def _central_solver(self):
        """Rank 0's whole-mesh counterpart that runs the partitioned solver's updates (same arguments,
        no partition)."""
        return NavierStokesSolver(**self._args)

    def _get_update_partitioned(self, dres_u, dres_v, dres_cont, du0, dv0, dp0):
        """Whole-mesh update for a strip-partitioned solver: the linearisation (the residual's u, v for
        Sys, the Jacobian's u, v) and the right-hand sides are gathered; rank 0 hands them to its
        whole-mesh counterpart through the reference interface (_get_residuals sets Sys,
        _calc_jacobians the Jacobians, _get_update solves) and broadcasts the update."""
        part = self._part
        lin = self._lin
        if lin is None:
            raise RuntimeError("NavierStokes: _calc_jacobians must run before _get_update")
        stale = lin.get("stale")
        if stale:
            us, vs = (self._global(a) for a in lin["sys"])
            uj, vj = (self._global(a) for a in lin["jac"])
            lin["stale"] = False
        rhs = [self._global(a) for a in (dres_u, dres_v, dres_cont)]
        x0 = [None if a is None else self._global(a) for a in (du0, dv0, dp0)]
        out = torch.zeros(3 * self.N + 1, dtype=torch.float64)
        err = None
        if part.rank == 0:
            # a failure on rank 0 (non-convergence, a singular block, out of memory) travels in the
            # broadcast as a NaN status, so every rank raises instead of waiting in the collective
            try:
                if stale:
                    if self._twin is None:
                        self._twin = self._central_solver()
                    z = np.zeros(self.N)
                    self._twin._get_residuals(us, vs, z, z)
                    self._twin._calc_jacobians(uj, vj)
                d = self._twin._get_update(*rhs, du0=x0[0], dv0=x0[1], dp0=x0[2])
                out[:3 * self.N] = torch.from_numpy(np.concatenate([np.asarray(a) for a in d]))
                out[-1] = float(getattr(self._twin, "schur_matvecs", -1))
            except (RuntimeError, ValueError) as e:
                err = e
                out[-1] = float("nan")
        out = part.broadcast(out)
        if err is not None:
            raise err
        if torch.isnan(out[-1]):
            raise RuntimeError("NavierStokes: the update failed on rank 0 (see its error)")
        self.schur_matvecs = int(out[-1].item())
        d = [out[i * self.N:(i + 1) * self.N].cpu().numpy() for i in range(3)]
        if isinstance(dres_u, torch.Tensor):
            return tuple(self._dev(a) for a in d)
        return tuple(d)

    def _use_nd(self):
        """Nested dissection (velocity_interior "auto" / "nd") needs P >= 2 and the whole perimeter Dirichlet."""
        ok = self._P >= 2 and self._dir.mask is None and self._dir.sides == _ALL_SIDES
        if self._velocity_interior == "nd" and not ok:
            raise ValueError("velocity_interior='nd' needs P >= 2 and the whole perimeter Dirichlet")
        return ok and self._velocity_interior in ("auto", "nd")

    def _strip_velocity_solver(self):
        """The element-partitioned velocity factor of this linearisation on this rank's strip handle
        (nested_dissection.StripNDSolver, or strip_solve.StripLineSolver for other Dirichlet sets), kept until
        _calc_jacobians runs again."""
        if self._velo is not None:
            return self._velo
        from .nested_dissection import StripNDSolver
        from .strip_solve import StripLineSolver
        tStart = time.perf_counter()
        m, p = self._mesh, self._part
        # every rank takes the same choice: the Dirichlet set and the option are global
        cls = StripNDSolver if self._use_nd() else StripLineSolver
        vs = cls(self._P, self._N_ex, self._N_ey, m.device, p.part.bounds, p.rank, p.dist, group=p.group,
                 gather_device=p.backend_device())
        vs.factor_mesh(m, dir_mask=self._dir.mask, dir_sides=self._dir.sides, **self._jac_kw)
        vs.set_operator(self._velocity_apply_lines, amax=lambda t: p.amax(t))
        vs.check_refinement()       # every rank takes the same decision (norms max-reduced over the ranks)
        self._velo = vs
        if 'LU_suc' in self._iprint:
            print(f'NavierStokes LU: Succeeded in {time.perf_counter()-tStart:0.2f}sec (element-partitioned)')
        return vs

    def _schur_strips(self, vs, dp):
        """S dp on the strips (NavierStokes_Solver.py:194-203): the gradients of dp (interface lines summed
        across strips), the partitioned velocity solve, the divergence (summed)."""
        m, part, NY = self._mesh, self._part, self._mesh.NY
        kw = self._ns_kw(pin_first=False)
        gu, gv = torch.empty_like(dp), torch.empty_like(dp)
        with phase("schur.grad_apply"):
            m.ns_apply(None, None, dp, gu, gv, **kw)
        with phase("schur.grad_assemble"):
            part.assemble(gu, gv)
        with phase("schur.velocity_solve"):
            X = vs._solve_lines(torch.stack((gu.view(-1, NY), gv.view(-1, NY)), dim=1).reshape(-1, 2 * NY))
        rc = torch.empty_like(dp)
        with phase("schur.div_apply"):
            m.ns_apply(X[:, :NY].reshape(-1), X[:, NY:].reshape(-1), dp, rc=rc, c_div=-1.0, **kw)
        with phase("schur.div_assemble"):
            part.assemble(rc)
        return rc

    def _get_update_strips(self, dres_u, dres_v, dres_cont, du0=None, dv0=None, dp0=None):
        """_get_update (NavierStokes_Solver.py:162-236) on the strips: the element-partitioned velocity
        solve inside the Schur-complement GMRES, whose inner products are all-reduced (a shared line
        counted once); the reference's mass-diagonal preconditioner and stopping rule."""
        vs = self._strip_velocity_solver()
        m, part = self._mesh, self._part
        kw = self._ns_kw(pin_first=False)
        ru, rv, rc = self._dev(dres_u), self._dev(dres_v), self._dev(dres_cont)
        fu, fv = vs.solve(ru, rv)
        c0 = torch.empty_like(rc)
        m.ns_apply(fu, fv, None, rc=c0, **kw)
        part.assemble(c0)
        b_schur = rc - c0
        count = [0]
        if self._schur is None:
            self._schur = _StripSchur(self, vs, graph=self._velocity_graph)

        def schur_mv(dp):
            count[0] += 1
            return self._schur(dp)

        pin = self._pin_local

        def precon(c):
            z = c / self._Mdiag
            if pin >= 0:
                z[pin] = c[pin]
            return z

        it = [0]
        prog = getattr(self, "_progress", 0)
        t_start = time.perf_counter()

        def cb(est):
            it[0] += 1
            if 'LGMRES_iter' in self._iprint or (prog and it[0] % prog == 0):
                print(f'NavierStokes GMRES: {it[0]}\t{est}\t{time.perf_counter() - t_start:.1f}s', flush=True)

        # restart and maxiter from sizes every rank shares (the largest strip, the global N): the ranks
        # run the same Arnoldi iterations and so call the same collectives
        restart = max(1, min(self.N, self._max_basis, int(32e9 // (16 * part.max_local_dofs()))))
        r = gmres(schur_mv, b_schur, x0=self._dev(dp0), atol=self._mtol * np.sqrt(self.N), rtol=0.0,
                  restart=restart, maxiter=10 * self.N, precond=precon, callback=cb, inner=part.inner)
        if r.info != 0:
            raise RuntimeError(f'NavierStokes LGMRES: Failed to converge in {r.info} iterations')
        dp = r.x
        self.schur_matvecs = count[0] - r.discarded     # a dropped speculative matvec is not counted
        self.schur_discarded = r.discarded
        b_u, b_v = torch.empty_like(dp), torch.empty_like(dp)
        m.ns_apply(None, None, dp, b_u, b_v, **kw)
        part.assemble(b_u, b_v)
        du, dv = vs.solve(ru - b_u, rv - b_v)
        return self._out(du, dres_u), self._out(dv, dres_u), self._out(dp, dres_u)

    def _velocity_solver(self):
        """Device factorisation of the Dirichlet-row-replaced velocity Jacobian -- the reference's
        `bmat` + `splu` (NavierStokes_Solver.py:176-184) -- by static condensation over node lines
        (sem_amd/solvers/velocity_solve.py).  The reference refactorises on every _get_update call;
        the factor depends only on the Jacobians, so it is kept until _calc_jacobians runs again (the
        Boussinesq coupler's block-Jacobi preconditioner calls _get_update once per Krylov iteration)."""
        if self._velo is not None:
            return self._velo
        tStart = time.perf_counter()
        m = self._mesh
        if self.N > 1_000_000:   # the previous linearisation's factor and graphs go before the next one
            gc.collect()
            torch.cuda.empty_cache()
        interior = self._velocity_interior
        if self._use_nd():
            # nested dissection of the element grid (solvers/nested_dissection.py): cfg5 3.0 ms per solve with the
            # split leaves against the line condensation's 7.8 ms, cfg4 0.34 against 0.56 ms (profiles/r06/velocity/)
            vs = NestedDissectionSolver(self._P, self._N_ex, self._N_ey, m.device)
        else:
            vs = VelocityJacobianSolver(self._P, self._N_ex, self._N_ey, m.device,
                                        interior="nested" if interior == "auto" else interior, sweep=self._velocity_sweep)
        vs.factor_mesh(m, dir_mask=self._dir.mask, dir_sides=self._dir.sides, **self._jac_kw)
        vs.set_operator(self._velocity_apply_lines)
        vs.check_refinement()       # one refinement step per solve if the factor's backward error exceeds 1e-13
        if self._velocity_graph:
            vs.capture()
        self._velo = vs
        if 'LU_suc' in self._iprint:
            torch.cuda.synchronize(m.device)
            kind = ("nested dissection" + (", split leaves" if vs.split else ", A_ii^-1 leaves")
                    if vs.interior == "nd" else "device static condensation")
            print(f'NavierStokes LU: Succeeded in {time.perf_counter()-tStart:0.2f}sec ({kind}, '
                  f'backward error {vs.refine_eta:.1e}{", refined" if vs.refine else ""})')
        return vs

    def _velocity_apply_lines(self, X):
        """J X for the velocity Jacobian of this linearisation on (NX, 2 NY) line arrays: the velocity rows of
        _get_dresiduals at dp = 0 (NavierStokes_Solver.py:138-160; Dirichlet rows identity, as the factored
        Jacobian's), assembled across strips on a partitioned solver.  The refinement step's operator."""
        m, NY = self._mesh, self._mesh.NY
        kw = dict(self._jac_kw, **self._ns_kw(pin_first=False))
        if self._part is None:
            Y = torch.empty_like(X)
            m.ns_apply(X[:, :NY], X[:, NY:], None, Y[:, :NY], Y[:, NY:], None, **kw)
            return Y
        xu, xv = X[:, :NY].reshape(-1), X[:, NY:].reshape(-1)
        ru, rv = torch.empty_like(xu), torch.empty_like(xv)
        m.ns_apply(xu, xv, None, ru, rv, None, **kw)
        self._part.assemble(ru, rv)
        return torch.stack((ru.view(-1, NY), rv.view(-1, NY)), dim=1).reshape(-1, 2 * NY)

    def _pressure_laplacian(self):
        """A_p = K with the pinned pressure row as an identity row (the Neumann pressure Laplacian
        made regular), factored once per solver by the one-component line condensation."""
        if self._Ap is None:
            m = self._mesh
            vs = VelocityJacobianSolver(self._P, self._N_ex, self._N_ey, m.device, ncomp=1)
            mask = torch.zeros(m.n_local, dtype=torch.uint8, device=m.device)
            mask[self._pin if self._pin >= 0 else self.N // 2] = 1
            vs.factor_mesh(m, c_stiff=1.0, dir_mask=mask)
            if self._velocity_graph and m.device.type == "cuda":
                vs.capture()
            self._Ap = vs
        return self._Ap

    def _pcd(self, c):
        """z = A_p^-1 (F_p (w c) + b c): w = 1/M on continuity rows (0 elsewhere), b = 1 on the
        replaced rows (boundary K rows and the pin), F_p = Sys of this linearisation."""
        y = self._mesh.apply(c * self._pcd_w, **{k: self._jac_kw[k] for k in ("c_stiff", "c_mass", "c_gradx", "cu",
                                                                              "c_grady", "cv")},
                             c_extra=1.0, ea=c, eb=self._pcd_b)
        return self._pressure_laplacian().solve1(y)

    def _get_update(self, dres_u, dres_v, dres_cont, du0=None, dv0=None, dp0=None):
        """Velocity solve + pressure Schur-complement Krylov solve (NavierStokes_Solver.py:162-236), on
        the device: the velocity Jacobian is factored once per linearisation (_velocity_solver) and the
        Schur system is solved by the device GMRES (sem_amd/krylov.py) with the reference's
        mass-diagonal preconditioner (:208-212) and stopping rule ||r||_2 <= mtol sqrt(N) (:222-224).
        The reference's inner_m = 0.3 N is "not a realistic inner_m" (:224): its LGMRES runs as an
        unrestarted GMRES with outer augmentation.  A plain GMRES restarted at 0.3 N stagnates on small
        meshes (the Schur complement carries the spurious pressure modes of the equal-order
        discretisation), so the device GMRES runs unrestarted up to max_basis vectors."""
        if self._part is not None:
            if self._partition_update == "central":
                return self._get_update_partitioned(dres_u, dres_v, dres_cont, du0, dv0, dp0)
            return self._get_update_strips(dres_u, dres_v, dres_cont, du0, dv0, dp0)
        vs = self._velocity_solver()
        m = self._mesh
        ru, rv, rc = self._dev(dres_u), self._dev(dres_v), self._dev(dres_cont)
        fu, fv = vs.solve(ru, rv)
        c0 = torch.empty_like(rc)
        m.ns_apply(fu, fv, None, rc=c0, **self._ns_kw(pin_first=False))   # dres_cont(J^-1 [ru; rv], 0)
        b_schur = rc - c0
        if self._schur is None:
            self._schur = _SchurComplement(self, vs, graph=self._velocity_graph)
        count = [0]

        def schur_mv(dp):
            count[0] += 1
            return self._schur(dp)

        pin = self._pin

        def precon(c):
            z = c / self._Mdiag
            if pin >= 0:
                z[pin] = c[pin]
            return z

        if self._schur_precond == "pcd":
            precon = self._pcd

        it = [0]

        prog = getattr(self, "_progress", 0)

        def cb(est):
            it[0] += 1
            if 'LGMRES_iter' in self._iprint or (prog and it[0] % prog == 0):
                print(f'NavierStokes GMRES: {it[0]}\t{est}', flush=True)

        # the basis and its preconditioned images (2 restart N doubles = 16 N bytes per vector) within
        # 32 GB: unrestarted up to max_basis on cfg3/cfg4, restarted at 846 vectors on a whole-mesh cfg5
        # solver (N = 1537^2 = 2.36 M; 31.9 GB).  The velocity factor, the Schur graph's buffers and
        # the Hessenberg matrix come on top of this budget.
        # restart within 16 bytes per DOF per vector (847 at cfg5): twice that (V only, as krylov.gmres keeps no
        # M^-1 V for the linear mass-diagonal preconditioner) measured no faster at cfg5 -- fewer iterations in the
        # long first solves, each dearer (profiles/r04/cfg5/cfg5_restart1694.json)
        restart = max(1, min(self.N, self._max_basis, int(32e9 // (16 * self.N))))
        if self._recycle_bytes and self._schur_recycle is None:
            cap = min(self.N, max(restart + 1, int(self._recycle_bytes // (16 * self.N))))
            self._schur_recycle = Recycle(self.N, torch.float64, self._mesh.device, cap)
        r = gcro(schur_mv, b_schur, x0=self._dev(dp0), atol=self._mtol * np.sqrt(self.N), rtol=0.0,
                 restart=restart, precond=precon, callback=cb, recycle=self._schur_recycle)
        if r.info != 0:
            raise RuntimeError(f'NavierStokes LGMRES: Failed to converge in {r.info} iterations')
        dp = r.x
        self.schur_matvecs = count[0] - getattr(r, "discarded", 0)   # dropped speculations are not counted
        self.schur_discarded = getattr(r, "discarded", 0)
        if 'LGMRES_suc' in self._iprint:
            res = (schur_mv(dp) - b_schur).abs().max().item()
            print(f'NavierStokes GMRES: Converged in {self.schur_matvecs} evaluations with max-norm {res}')
        b_u, b_v = torch.empty_like(dp), torch.empty_like(dp)
        m.ns_apply(None, None, dp, b_u, b_v, **self._ns_kw(pin_first=False))
        du, dv = vs.solve(ru - b_u, rv - b_v)
        return self._out(du, dres_u), self._out(dv, dres_u), self._out(dp, dres_u)

    def _get_solution(self, T, u0=None, v0=None, p0=None):
        """Newton iteration (NavierStokes_Solver.py:238-270), iterates kept on the device; NumPy in,
        NumPy out (device tensors in, device tensors out)."""
        like = T
        Z = torch.zeros(self._mesh.n_local, dtype=torch.float64, device=self._mesh.device)
        u = self._dev(u0) if u0 is not None else Z.clone()
        v = self._dev(v0) if v0 is not None else Z.clone()
        p = self._dev(p0) if p0 is not None else Z.clone()
        T = self._dev(T)
        self._k = 0
        self.newton_history = []
        while True:
            res_u, res_v, res_cont = self._get_residuals(u, v, p, T)
            norm = self._norm(res_u, res_v, res_cont)
            if 'NEWTON_iter' in self._iprint:
                print(f'NavierStokes NEWTON: {self._k}\t{norm}')
            if norm <= self._mtol_newton * np.sqrt(self.N * 3):
                self.newton_history.append((norm, 0))
                if 'NEWTON_suc' in self._iprint:
                    mx = self._amax(res_u, res_v, res_cont)
                    print(f'NavierStokes NEWTON: Converged in {self._k} iterations with max-norm {mx}')
                break
            self._calc_jacobians(u, v)
            du, dv, dp = self._get_update(-res_u, -res_v, -res_cont)
            self.newton_history.append((norm, self.schur_matvecs))
            u = u + du
            v = v + dv
            p = p + dp
            self._k += 1
        return self._out(u, like), self._out(v, like), self._out(p, like)

    def _get_vector(self, f_func):
        return f_func(self.points[0], self.points[1])

    def _get_interpol(self, f, points_plot):
        f_e = SEM.scatter(f, self._P, self._N_ex, self._N_ey)
        return SEM.eval_interpolation(f_e, self.points_e, points_plot)

    def run(self, T_func, points_plot):
        T = self._get_vector(T_func)
        u, v, p = self._get_solution(T)
        return self._get_interpol(u, points_plot), self._get_interpol(v, points_plot), self._get_interpol(p,
                                                                                                         points_plot)


class _StripSchur:
    """The strip-partitioned Schur-complement operator (_schur_strips: gradient launch + interface assembly,
    the element-partitioned velocity solve with its all-gather, divergence launch + assembly).  Under RCCL
    every step stays on the device (collectives included), so the whole matvec is captured in one hipGraph
    per linearisation, as the whole-mesh _SchurComplement is; the capture is used only after its replay has
    reproduced the eager matvec on a probe vector, and every rank takes the same decision.  Under gloo (the
    CPU rehearsal, host-staged collectives) the matvec stays eager."""

    def __init__(self, ns, vs, graph=True):
        self.ns, self.vs = ns, vs
        m, part = ns._mesh, ns._part
        self._graph = None
        # SEM_STRIP_GRAPH=0 keeps the matvec eager (the capture of RCCL collectives is checked against
        # the eager matvec on a probe vector, but no multi-GPU run has exercised it yet -- DESIGN.md section 7)
        if (graph and m.device.type == "cuda" and part.backend_device().type == "cuda"
                and os.environ.get("SEM_STRIP_GRAPH", "1") != "0"):
            self._capture()

    def _capture(self):
        ns, m, part = self.ns, self.ns._mesh, self.ns._part
        dev = m.device
        g0 = torch.Generator(device=dev).manual_seed(5)
        probe = torch.rand(m.n_local, dtype=torch.float64, device=dev, generator=g0)
        self._x = torch.zeros_like(probe)
        cur = torch.cuda.current_stream(dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            want = ns._schur_strips(self.vs, probe)   # warm-up outside the capture (workspaces, communicators)
        cur.wait_stream(s)
        g = torch.cuda.CUDAGraph()
        try:   # a capture executes no collective, so a rank whose capture fails cannot desynchronise the others
            with no_gc(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._out = ns._schur_strips(self.vs, self._x)
            ok = 1.0
        except RuntimeError:
            torch.cuda.synchronize(dev)
            ok = 0.0
        if self._agree(ok):    # every rank captured: replay (its collectives need every rank) and compare
            self._x.copy_(probe)
            g.replay()
            err = (self._out - want).abs().max() / want.abs().max().clamp(min=1e-300)
            if self._agree(1.0 if bool(err <= 1e-12) else 0.0):
                self._graph = g

    def _agree(self, ok):
        """True when every rank reports ok (one all-reduce)."""
        part = self.ns._part
        flag = torch.tensor([ok], dtype=torch.float64, device=self.ns._mesh.device)
        part.dist.all_reduce(flag, op=part.dist.ReduceOp.MIN, group=part.group)
        return float(flag.item()) == 1.0

    def __call__(self, dp):
        if self._graph is None:
            return self.ns._schur_strips(self.vs, dp)
        self._x.copy_(dp)
        self._graph.replay()
        return self._out.clone()


class _SchurComplement:
    """The pressure Schur-complement operator of _get_update (NavierStokes_Solver.py:194-203):
    S dp = dres_cont(-J^-1 [G_x dp; G_y dp]_D, dp), i.e. two fused sem_ns_apply launches around one
    velocity solve.  The gradients are written straight into the solve's line-interleaved [u | v]
    layout and the divergence reads the solution from it (uv_pitch = 2 N_y), and the whole matvec is
    captured in one hipGraph per linearisation: a Krylov iteration then costs one graph launch."""

    def __init__(self, ns, vs, graph=True):
        self.ns, self.vs = ns, vs
        m = ns._mesh
        self._B = torch.zeros((m.NX, 2 * m.NY), dtype=torch.float64, device=m.device)
        self._x = torch.zeros(m.n_local, dtype=torch.float64, device=m.device)
        self._graph = None
        if graph and m.device.type == "cuda" and (vs.P == 1 or vs.interior != "lu"):
            self._capture()

    def _body(self, dp):
        ns, m, NY = self.ns, self.ns._mesh, self.ns._mesh.NY
        B = self._B
        m.ns_apply(None, None, dp, B[:, :NY], B[:, NY:], **ns._ns_kw(pin_first=False))
        X = self.vs._solve_lines(B)
        rc = torch.empty_like(dp)
        m.ns_apply(X[:, :NY], X[:, NY:], dp, rc=rc, c_div=-1.0, **ns._ns_kw(pin_first=False))
        return rc

    def _capture(self):
        dev = self.ns._mesh.device
        cur = torch.cuda.current_stream(dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(cur)
        try:
            with torch.cuda.stream(s):
                self._body(self._x)   # warm-up outside the capture (library workspaces)
            cur.wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with no_gc(), torch.cuda.graph(g):
                self._out = self._body(self._x)
            self._graph = g
        except RuntimeError:
            torch.cuda.synchronize(dev)
            self._graph = None

    def __call__(self, dp):
        if self._graph is None:
            return self._body(dp)
        self._x.copy_(dp)
        self._graph.replay()
        return self._out.clone()
