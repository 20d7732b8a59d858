"""Convection-diffusion solver counterpart on the device operators.

Mirrors Solvers/ConvectionDiffusion_Solver.py:9-203 (same constructor, same
private methods the OpenMDAO component calls, same error behaviour), with the
operator applies on the GPU:

  * `_get_residuals`  (:73-92)   -> ONE fused launch: Sys T with Dirichlet rows
                                    res = T - T_dir (SEM_DIR_IDENTITY + dir_val)
  * `_calc_jacobians` (:94-102)  -> Pe*G_x T, Pe*G_y T once per linearisation
  * `_get_dresiduals` (:104-121) -> ONE fused launch: Sys dT + (Pe G_x T).du
                                    + (Pe G_y T).dv with Dirichlet rows dres = dT

Vectors may be NumPy arrays (returned as NumPy, like the reference) or float64
device tensors (kept on the device).  The Dirichlet mask is built exactly as the
reference builds it (np.isclose on the node coordinates, :62-71); when it is the
plain boundary-line set the kernel derives it from geometry (no mask traffic).
`_get_update` runs a device-resident GMRES (sem_amd/krylov.py: Krylov basis in
HBM, CGS2 orthogonalisation as GEMVs, same stopping rule atol = mtol*sqrt(N) as
the reference's LGMRES); `krylov="scipy"` keeps the reference's host LGMRES
around device matvecs.  On a whole-mesh solver the GMRES is right-preconditioned
by a direct solve of the Jacobian itself (`precond="condensed"`, the default):
the static condensation over node lines of the NS velocity solve
(velocity_solve.py) with one unknown per node, factored once per Sys.  Right
preconditioning leaves the stopping test on the true residual ||dres_op(dT) -
dres||_2, so the reference's rule is unchanged; the Krylov count drops from
hundreds-thousands of matvecs to one or two.
"""
import typing

import numpy as np
import scipy.sparse.linalg as linalg
import torch

from .. import SEM, _lib
from ..device import get_mesh
from ..krylov import Recycle, gcro, gmres
from ..operators import ConvectionTensor, SEMOperator
from .velocity_solve import VelocityJacobianSolver


def side_mask(points, L_x, L_y, sides):
    """Boundary-line mask for side bits, from the same np.isclose tests as the reference."""
    m = np.zeros(points.shape[1], dtype=bool)
    if sides & _lib.SIDE_W:
        m |= np.isclose(points[0], 0)
    if sides & _lib.SIDE_E:
        m |= np.isclose(points[0], L_x)
    if sides & _lib.SIDE_S:
        m |= np.isclose(points[1], 0)
    if sides & _lib.SIDE_N:
        m |= np.isclose(points[1], L_y)
    return m


def geometric_mask(NX, NY, sides):
    gx, gy = np.divmod(np.arange(NX * NY), NY)
    m = np.zeros(NX * NY, dtype=bool)
    if sides & _lib.SIDE_W:
        m |= gx == 0
    if sides & _lib.SIDE_E:
        m |= gx == NX - 1
    if sides & _lib.SIDE_S:
        m |= gy == 0
    if sides & _lib.SIDE_N:
        m |= gy == NY - 1
    return m


class DirichletRows:
    """Device form of a reference Dirichlet mask (global, np.isclose-built): side bits when it is
    exactly the boundary lines (the usual case), an explicit uint8 mask otherwise.  On a strip
    mesh the mask is the strip's slice."""

    def __init__(self, mesh, mask, sides):
        sl = slice(mesh.dof_begin, mesh.dof_begin + mesh.n_local)
        full = np.asarray(mask, dtype=bool)
        self.mask_np = full[sl]
        if np.array_equal(full, geometric_mask(mesh.NX, mesh.NY, sides)):
            self.sides, self.mask = sides, None
        else:
            self.sides = 0
            self.mask = torch.as_tensor(self.mask_np.astype(np.uint8), device=mesh.device)

    def kw(self):
        return dict(dir_sides=self.sides, dir_mask=self.mask)


class ConvectionDiffusionSolver:
    def __init__(self, L_x: float, L_y: float, Pe: float, P: int, N_ex: int, N_ey: int,
                 T_W: float = None, T_E: float = None, T_S: float = None, T_N: float = None,
                 mtol=1e-7, iprint: list = [], krylov: str = "device", max_basis: int = 2000,  # noqa: B006
                 partition=None, recycle_bytes: float = 0.0, precond: str = "condensed",
                 partition_update: str = "distributed"):
        """partition: a sem_amd.parallel.Partition -- the solver then holds one element-column strip
        per rank, every apply ends with the interface exchange (overlapped with the interior) and
        the Krylov inner products are all-reduced; the reference methods still take and return
        global NumPy vectors (local strips when given device tensors).
        partition_update: how a partitioned solver solves its Newton update -- "distributed": the
        device GMRES over the strips (every matvec a strip apply + exchange, inner products
        all-reduced), right-preconditioned by the element-partitioned condensed direct solve of the
        Jacobian (strip_solve.StripLineSolver: each rank factors its own columns, the ranks share a
        reduced system over the strip-boundary lines); "central": the Sys velocity field and the
        right-hand side are gathered, rank 0's whole-mesh counterpart (_central_solver) solves with
        the condensed direct preconditioner, the update is broadcast."""
        if krylov not in ("device", "scipy"):
            raise ValueError("krylov must be 'device' or 'scipy'")
        if partition is not None and krylov != "device":
            raise ValueError("a partitioned solver needs krylov='device'")
        if precond not in ("condensed", None):
            raise ValueError("precond must be 'condensed' or None")
        # a partitioned solver preconditions with the element-partitioned condensation (strip_solve.py)
        self._precond = precond
        if partition_update not in ("distributed", "central"):
            raise ValueError("partition_update must be 'distributed' or 'central'")
        self._partition_update = partition_update
        self._args = dict(L_x=L_x, L_y=L_y, Pe=Pe, P=P, N_ex=N_ex, N_ey=N_ey, T_W=T_W, T_E=T_E, T_S=T_S, T_N=T_N,
                          mtol=mtol, iprint=iprint, max_basis=max_basis, precond=precond)
        self._twin, self._sys_uv, self._twin_stale = None, None, True
        self._factor = None     # condensed Jacobian of the current Sys (rebuilt after _get_residuals)
        self._krylov, self._max_basis = krylov, max_basis
        self._part = partition
        # recycled Krylov subspace across _get_update calls with one operator (sem_amd.krylov.Recycle):
        # the Boussinesq coupler's block-Jacobi preconditioner solves with the same Sys tens of times
        self._recycle_bytes, self._recycle = recycle_bytes, None
        self._iprint = iprint
        self._Pe = Pe
        self._mtol = mtol
        self._L_x, self._L_y = L_x, L_y
        self._P, self._N_ex, self._N_ey = P, N_ex, N_ey
        dx, dy = L_x / N_ex, L_y / N_ey
        self.points = SEM.global_nodes(P, N_ex, N_ey, L_x / N_ex, L_y / N_ey)
        self.points_e = SEM.element_nodes(P, N_ex, N_ey, dx, dy)
        self.N = (N_ex * P + 1) * (N_ey * P + 1)
        if partition is None:
            self._mesh = get_mesh(P, N_ex, N_ey, dx, dy)
            self._apply = self._mesh.apply
        else:
            self._mesh = partition.setup(P, N_ex, N_ey, dx, dy)
            self._apply = partition.step

        # global operators (matrix-free; on a strip mesh when partitioned)
        m = self._mesh
        self._M = SEMOperator(m, cM=1.0)
        self._K = SEMOperator(m, cK=1.0)
        self._C_x, self._C_y = ConvectionTensor(m, "x"), ConvectionTensor(m, "y")
        self._Sys = None
        self._Jac_T_u = None
        self._Jac_T_v = None

        # Dirichlet values and mask (ConvectionDiffusion_Solver.py:62-71)
        self._dirichlet = np.full(self.N, np.nan)
        sides = 0
        for val, coord, target, bit in ((T_W, 0, 0, _lib.SIDE_W), (T_E, 0, L_x, _lib.SIDE_E),
                                        (T_S, 1, 0, _lib.SIDE_S), (T_N, 1, L_y, _lib.SIDE_N)):
            if val is not None:
                self._dirichlet[np.isclose(self.points[coord], target)] = val
                sides |= bit
        self._mask_dir = ~np.isnan(self._dirichlet)
        self._dir = DirichletRows(self._mesh, self._mask_dir, sides)
        self._dir_val = self._dev(np.where(self._mask_dir, self._dirichlet, 0.0))

    # ------------------------------------------------------------------ helpers
    def _dev(self, a):
        """Device vector of this solver's (local) DOFs; a global NumPy vector is sliced to the strip."""
        if a is None:
            return None
        if self._part is not None and not isinstance(a, torch.Tensor):
            a = self._part.local(np.asarray(a))
        return self._mesh.to_device(a)

    def _out(self, y, like):
        if isinstance(like, torch.Tensor):
            return y
        if self._part is not None:
            y = self._part.gather(y)
        return y.cpu().numpy()

    # ------------------------------------------------------------------ reference methods
    def _get_residuals(self, T, u, v):
        """res = Sys T, Dirichlet rows T - T_dir (ConvectionDiffusion_Solver.py:73-92)."""
        Conv = self._Pe * (SEM.tensordot(self._C_x, self._dev(u), (1, 0)) + SEM.tensordot(self._C_y, self._dev(v), (1, 0)))
        self._Sys = Conv + self._K
        self._factor = None
        if self._part is not None:
            self._sys_uv, self._twin_stale = (self._dev(u), self._dev(v)), True
        if self._recycle is not None:   # the update operator depends on Sys
            self._recycle.reset()
        y = self._apply(self._dev(T), dir_mode=_lib.DIR_IDENTITY, dir_val=self._dir_val, **self._sys_kw(),
                        **self._dir.kw())
        return self._out(y, T)

    def _sys_kw(self):
        cX, cu, cY, cv, d = self._Sys._coeffs()
        return dict(c_stiff=self._Sys.cK, c_mass=self._Sys.cM, c_gradx=cX, cu=cu, c_grady=cY, cv=cv)

    def _calc_jacobians(self, T):
        """Pe diag(G_x T), Pe diag(G_y T) (ConvectionDiffusion_Solver.py:94-102)."""
        if self._part is None:
            self._Jac_T_u = self._Pe * SEM.tensordot(self._C_x, T, (2, 0))
            self._Jac_T_v = self._Pe * SEM.tensordot(self._C_y, T, (2, 0))
        else:  # G_x T on a strip needs the interface exchange before it becomes a diagonal
            Td = self._dev(T)
            self._Jac_T_u = SEMOperator(self._mesh, dg=[(self._Pe, self._apply(Td, c_gradx=1.0))])
            self._Jac_T_v = SEMOperator(self._mesh, dg=[(self._Pe, self._apply(Td, c_grady=1.0))])

    def _get_dresiduals(self, dT, du=None, dv=None):
        """dres = Sys dT + J_u du + J_v dv, Dirichlet rows dT (ConvectionDiffusion_Solver.py:104-121)."""
        kw = {}
        if du is not None or dv is not None:
            ju = self._Jac_T_u._coeffs()[4] if du is not None else None
            jv = self._Jac_T_v._coeffs()[4] if dv is not None else None
            kw = dict(c_extra=1.0, ea=ju, eb=self._dev(du), ec=jv, ed=self._dev(dv))
        y = self._apply(self._dev(dT), dir_mode=_lib.DIR_IDENTITY, **self._sys_kw(), **self._dir.kw(), **kw)
        return self._out(y, dT)

    def _get_update(self, dres, dT0=None):
        """Newton update: solve dres_op(dT) = dres (ConvectionDiffusion_Solver.py:123-156)."""
        if self._part is not None and self._partition_update == "central":
            return self._get_update_central(dres, dT0)
        if self._krylov == "device":
            return self._get_update_device(dres, dT0)
        return self._get_update_scipy(dres, dT0)

    def _jacobian_solver(self):
        """Direct solve of dres_op = Sys with Dirichlet identity rows (ConvectionDiffusion_Solver.py:
        104-121 at du = dv = 0): sem_condensed_blocks with one component writes the condensation
        pieces, VelocityJacobianSolver factors them (on a partitioned solver: StripLineSolver, each rank
        its own strip); kept until Sys changes (_get_residuals)."""
        if self._factor is None:
            if self._Sys is None:
                raise RuntimeError("ConvectionDiffusion: _get_residuals must run before _get_update")
            m = self._mesh
            if self._part is not None:
                from .strip_solve import StripLineSolver
                p = self._part
                vs = StripLineSolver(self._P, self._N_ex, self._N_ey, m.device, p.part.bounds, p.rank, p.dist,
                                     group=p.group, ncomp=1, gather_device=p.backend_device())
            else:
                vs = VelocityJacobianSolver(self._P, self._N_ex, self._N_ey, m.device, ncomp=1)
            cX, cu, cY, cv, d = self._Sys._coeffs()
            vs.factor_mesh(m, c_mass=self._Sys.cM, c_stiff=self._Sys.cK, c_gradx=cX, cu=cu, c_grady=cY, cv=cv, juu=d,
                           **self._dir.kw())
            if m.device.type == "cuda":
                vs.capture()
            self._factor = vs
        return self._factor

    def _get_update_device(self, dres, dT0=None):
        """GMRES with the Krylov basis in HBM; restart = min(int(0.3 N), max_basis) (the
        reference's inner_m, capped so the basis fits device memory), right-preconditioned by the
        condensed direct solve when precond="condensed"."""
        b = self._dev(dres)
        x0 = self._dev(dT0)
        it = [0]

        prog = getattr(self, "_progress", 0)

        def cb(est):
            it[0] += 1
            if "LGMRES_iter" in self._iprint or (prog and it[0] % prog == 0):
                print(f"ConvectionDiffusion GMRES: {it[0]}\t{est}", flush=True)

        restart = max(1, min(int(self.N * 0.3), self._max_basis))
        precond = None
        if self._precond == "condensed" and (self._part is None or self._P > 1):
            precond = self._jacobian_solver().solve1
            restart = min(restart, 100)
        if self._part is not None:
            r = gmres(lambda v: self._get_dresiduals(v), b, x0=x0, atol=self._mtol * np.sqrt(self.N), rtol=0.0,
                      restart=restart, maxiter=10 * self.N, precond=precond, callback=cb, inner=self._part.inner)
        else:
            if self._recycle_bytes and self._recycle is None:
                n = self._mesh.n_local
                cap = min(n, max(restart + 1, int(self._recycle_bytes // (16 * n))))
                self._recycle = Recycle(n, torch.float64, self._mesh.device, cap)
            r = gcro(lambda v: self._get_dresiduals(v), b, x0=x0, atol=self._mtol * np.sqrt(self.N), rtol=0.0,
                     restart=restart, precond=precond, callback=cb,
                     recycle=self._recycle if precond is None else None)
        if r.info != 0:
            raise RuntimeError(f"ConvectionDiffusion LGMRES: Failed to converge in {r.info} iterations")
        self.matvecs = r.matvecs
        if "LGMRES_suc" in self._iprint:
            res = (self._get_dresiduals(r.x) - b).abs().max().item()
            print(f"ConvectionDiffusion GMRES: Converged in {r.matvecs} evaluations with max-norm {res}")
        return self._out(r.x, dres)

    def _central_solver(self):
        """Rank 0's whole-mesh counterpart for partition_update="central" (same arguments, no
        partition)."""
        return ConvectionDiffusionSolver(**self._args)

    def _global(self, a):
        if isinstance(a, torch.Tensor):
            return self._part.gather(a).cpu().numpy()
        return np.asarray(a, dtype=np.float64)

    def _get_update_central(self, dres, dT0=None):
        """The partitioned solver's update on rank 0's whole-mesh counterpart: its Sys is set from
        the gathered velocity field of the last _get_residuals (the reference interface), it solves
        with the condensed direct preconditioner, and the update is broadcast to every rank."""
        part = self._part
        if self._sys_uv is None:
            raise RuntimeError("ConvectionDiffusion: _get_residuals must run before _get_update")
        stale = self._twin_stale
        if stale:
            u, v = (self._global(a) for a in self._sys_uv)
            self._twin_stale = False
        b = self._global(dres)
        x0 = None if dT0 is None else self._global(dT0)
        out = torch.zeros(self.N + 1, dtype=torch.float64)
        err = None
        if part.rank == 0:
            try:   # a rank-0 failure is broadcast as a NaN status: every rank raises, none waits
                if stale:
                    if self._twin is None:
                        self._twin = self._central_solver()
                    self._twin._get_residuals(np.zeros(self.N), u, v)
                out[:self.N] = torch.from_numpy(np.asarray(self._twin._get_update(b, dT0=x0)))
                out[-1] = float(getattr(self._twin, "matvecs", -1))
            except (RuntimeError, ValueError) as e:
                err = e
                out[-1] = float("nan")
        out = part.broadcast(out)
        if err is not None:
            raise err
        if torch.isnan(out[-1]):
            raise RuntimeError("ConvectionDiffusion: the update failed on rank 0 (see its error)")
        self.matvecs = int(out[-1].item())
        dT = out[:self.N].cpu().numpy()
        return self._dev(dT) if isinstance(dres, torch.Tensor) else dT

    def _get_update_scipy(self, dres, dT0=None):
        """The reference's LGMRES on the host around device matvecs."""

        def lhs_mv(dT):
            lhs_mv.fCount += 1
            return self._get_dresiduals(np.ascontiguousarray(dT, dtype=np.float64).ravel())

        lhs_mv.fCount = 0
        lhs_LO = linalg.LinearOperator((self.N,) * 2, lhs_mv, dtype=float)
        dres = np.asarray(dres.cpu().numpy() if isinstance(dres, torch.Tensor) else dres)

        def print_res(xk):
            print_res.iterCount += 1
            if "LGMRES_iter" in self._iprint:
                print(f"ConvectionDiffusion LGMRES: {print_res.iterCount}\t{np.linalg.norm(lhs_LO.matvec(xk) - dres)}")

        print_res.iterCount = 0
        dT, info = linalg.lgmres(A=lhs_LO, b=dres, M=None, x0=dT0, atol=self._mtol * np.sqrt(self.N), rtol=0,
                                 inner_m=int(self.N * 0.3), callback=print_res)
        if info != 0:
            raise RuntimeError(f"ConvectionDiffusion LGMRES: Failed to converge in {info} iterations")
        if "LGMRES_suc" in self._iprint:
            res = np.linalg.norm(lhs_LO.matvec(dT) - dres, ord=np.inf)
            print(f"ConvectionDiffusion LGMRES: Converged in {lhs_mv.fCount} evaluations with max-norm {res}")
        return dT

    def _get_solution(self, u, v, T0=None):
        """Single Newton step (ConvectionDiffusion_Solver.py:158-170)."""
        if self._part is not None and not isinstance(u, torch.Tensor):   # strips for the whole step
            Tl = self._dev(T0) if T0 is not None else torch.zeros(self._mesh.n_local, dtype=torch.float64,
                                                                   device=self._mesh.device)
            Tl = self._get_solution(self._dev(u), self._dev(v), Tl)
            return self._out(Tl, u)
        T = T0 if T0 is not None else np.zeros(self.N)
        res = self._get_residuals(T, u, v)
        dT = self._get_update(-res)
        return T + dT

    def _get_vector(self, f_func: typing.Callable[[np.ndarray, np.ndarray], np.ndarray]) -> np.ndarray:
        return f_func(self.points[0], self.points[1])

    def _get_interpol(self, f, points_plot):
        f_e = SEM.scatter(f, self._P, self._N_ex, self._N_ey)
        return SEM.eval_interpolation(f_e, self.points_e, points_plot)

    def run(self, u_func, v_func, points_plot):
        u = self._get_vector(u_func)
        v = self._get_vector(v_func)
        T = self._get_solution(u, v)
        return self._get_interpol(T, points_plot)
