"""Boussinesq coupler counterpart: natural convection, NS + CD coupled.

Restates OpenMDAO/Boussinesq_SequentialCoupler.py:10-108 (and the arithmetic of
Boussinesq_ParallelCoupler.py:12-121, which differs only in where the two blocks run)
without OpenMDAO, which is not available offline.  The two OpenMDAO components
(OpenMDAO/ConvectionDiffusion_Component.py, OpenMDAO/NavierStokes_Component.py) are
restated as the residual / Jacobian / block-solve maps below.  Everything they call is a
solver counterpart (sem_amd.solvers), so every operator apply is a HIP kernel launch and
the CD Newton updates run the device GMRES.  Any pair of objects with the reference
solvers' private methods can be passed in (the golden fixture tests/golden/bous.npz was
made by this coupler driving the reference's own solver classes).

Coupled system (the PG group of the couplers, :66-73):
    R_cd(T; u, v)     = cd._get_residuals(T, I_cd(u), I_cd(v))          (output T_cd)
    R_ns(u, v, p; T)  = ns._get_residuals(u, v, p, I_ns(T))             (outputs u_ns, v_ns, p_ns)
where I_cd / I_ns are the mesh transfers of change_inputs (CD component :23-36, NS component
:23-33): the other solver's solution interpolated at this solver's nodes (the identity when
both meshes agree, which the coupler then skips).

Modes (:40-41,75-93):
    'JNK'  Newton; linear system by restarted GMRES (restart 20, atol = mtol_gmres*sqrt(DOF),
           rtol 0) preconditioned by one block-Jacobi sweep (each component's solve_linear:
           cd._get_update / ns._get_update).  OpenMDAO's ScipyKrylov hands the preconditioner
           to SciPy's GMRES as M, i.e. on the LEFT; krylov.gmres_left restates that algorithm
           (see its docstring for why the side matters here).  The block-Jacobi sweep is the
           block-diagonal solve: zero initial guesses, no off-diagonal terms (the coupler's
           comment says it "requires change in linear_block_jac.py"; the changed file is not
           in the reference, so this is the textbook block-Jacobi preconditioner).
    'NJ'   Newton whose linear solve is the block-Jacobi sweep alone, with an Armijo-Goldstein
           line search (maxiter AGi, contraction AGr, slope AGc).
    'GS'   nonlinear block Gauss-Seidel: CD solve, then NS solve, until the residual norm is
           below atol.
Newton starts as OpenMDAO's NewtonSolver(solve_subsystems=True, max_sub_solves=0) does: one
Gauss-Seidel pass of the subsystems' solve_nonlinear, then pure Newton steps.  Convergence is
||R||_2 <= mtol_nonlin * sqrt(DOF), DOF = 3 N_ns + N_cd (:61-63).
"""
import math
import time

import numpy as np
import torch

from ..krylov import gmres_left


class BoussinesqCoupler:
    def __init__(self, L_x, L_y, Re=1.e3, Ra=1.e3, Pr=0.71, P_cd=4, N_ex_cd=8, N_ey_cd=8, P_ns=4, N_ex_ns=8,
                 N_ey_ns=8, mode='JNK', mtol_nonlin=1e-9, AGi=8, AGr=0.8, AGc=0.2, mtol_gmres=1e-10, restart=20,
                 mtol_internal=1e-13, maxiter=None, iprint=0, cd=None, ns=None, schur_precond="mass"):
        """schur_precond: the NS solver's Schur-complement preconditioner ("mass" = the reference's,
        "pcd" = pressure convection-diffusion; NavierStokesSolver)."""
        if mode not in ('JNK', 'NJ', 'GS'):
            raise ValueError('Unknown method')
        self.mode, self.iprint = mode, iprint
        self.AGi, self.AGr, self.AGc, self.restart = AGi, AGr, AGc, restart
        # backend solvers exactly as the couplers build them (:52-59)
        if cd is None:
            from .convection_diffusion import ConvectionDiffusionSolver
            cd = ConvectionDiffusionSolver(L_x=L_x, L_y=L_y, Pe=Re * Pr, P=P_cd, N_ex=N_ex_cd, N_ey=N_ey_cd,
                                           T_W=0.5, T_E=-0.5, mtol=mtol_internal)
        if ns is None:
            from .navier_stokes import NavierStokesSolver
            ns = NavierStokesSolver(L_x=L_x, L_y=L_y, Re=Re, Gr=Ra / Pr, P=P_ns, N_ex=N_ex_ns, N_ey=N_ey_ns,
                                    mtol=mtol_internal, mtol_newton=mtol_internal, iprint=[],
                                    schur_precond=schur_precond)
        self.cd, self.ns = cd, ns
        self.Ncd, self.Nns = cd.N, ns.N
        self.DOF = 3 * self.Nns + self.Ncd
        self.atol_gmres = mtol_gmres * math.sqrt(self.DOF)
        self.atol_nonlin = mtol_nonlin * math.sqrt(self.DOF)
        self.maxiter = maxiter if maxiter is not None else {'JNK': 100, 'NJ': 1000, 'GS': 1000}[mode]
        self._same_mesh = (cd._P, cd._N_ex, cd._N_ey) == (ns._P, ns._N_ex, ns._N_ey)
        # device mode: the coupled vector lives on the device as [T | u | v | p] of this rank's strips (the
        # whole mesh when the solvers are not partitioned), the solver methods exchange device tensors, and
        # the coupled Krylov / Newton iteration runs there -- no host copy of the 4 N vectors per step, and
        # on a partition only the interface lines (inside the solver maps) and inner products cross ranks.
        # Reference solver classes (duck-typed, NumPy) keep the host mode.
        self._device = (getattr(cd, "_mesh", None) is not None and getattr(ns, "_mesh", None) is not None
                        and self._same_mesh)
        self._inner = None
        if self._device:
            self._ncd_loc, self._nns_loc = cd._mesh.n_local, ns._mesh.n_local
            pcd, pns = getattr(cd, "_part", None), getattr(ns, "_part", None)
            if (pcd is None) != (pns is None):
                raise ValueError("partition both solvers or neither")
            if pns is not None:
                # the owned ranges of [T | u | v | p]: each block's own strip range (a shared line counted once)
                from ..parallel import DistributedInner
                segs, off = [], 0
                for blk in (pcd.inner, pns.inner, pns.inner, pns.inner):
                    segs += [(off + a, off + b) for a, b in blk.segments]
                    off += blk.n
                self._inner = DistributedInner(None, (off, cd._mesh.device), pns.dist, pns.group, segments=segs,
                                               backend_device=pns.backend_device())
        self.iterations = 0
        self.timing = {k: 0.0 for k in ("residuals", "jacobian_apply", "cd_update", "ns_update")}
        self.calls = {k: 0 for k in self.timing}

    def _timed(self, key, fn, *a, **kw):
        t0 = time.perf_counter()
        r = fn(*a, **kw)
        self.timing[key] += time.perf_counter() - t0
        self.calls[key] += 1
        return r

    # ------------------------------------------------------------------ mesh transfers (change_inputs)
    def _to_cd(self, f_ns):
        """ConvectionDiffusion_Component.change_inputs (:23-36): NS field at the CD nodes."""
        if self._same_mesh:
            if isinstance(f_ns, torch.Tensor):
                return f_ns.clone()
            return np.array(f_ns, dtype=np.float64, copy=True)
        cd = self.cd
        shape = (2, cd._P * cd._N_ex + 1, cd._P * cd._N_ey + 1)
        return np.asarray(self.ns._get_interpol(f_ns, np.reshape(cd.points, shape))).flatten()

    def _to_ns(self, f_cd):
        """NavierStokes_Component.change_inputs (:23-33): CD field at the NS nodes."""
        if self._same_mesh:
            if isinstance(f_cd, torch.Tensor):
                return f_cd.clone()
            return np.array(f_cd, dtype=np.float64, copy=True)
        ns = self.ns
        shape = (2, ns._P * ns._N_ex + 1, ns._P * ns._N_ey + 1)
        return np.asarray(self.cd._get_interpol(f_cd, np.reshape(ns.points, shape))).flatten()

    # ------------------------------------------------------------------ packing
    def _split(self, x):
        n, m = (self._ncd_loc, self._nns_loc) if self._device else (self.Ncd, self.Nns)
        return x[:n], x[n:n + m], x[n + m:n + 2 * m], x[n + 2 * m:]

    def _join(self, *parts):
        if self._device:
            return torch.cat([a.reshape(-1) for a in parts])
        return np.concatenate([np.asarray(a, dtype=np.float64) for a in parts])

    def _norm(self, r):
        if not self._device:
            return np.linalg.norm(r)
        if self._inner is None:
            return torch.linalg.vector_norm(r).item()
        return math.sqrt(float(self._inner(r[None], r)[0]))

    def _zeros(self, n_global, n_local, like=None):
        if self._device:
            return torch.zeros(n_local, dtype=torch.float64, device=self.cd._mesh.device)
        return np.zeros(n_global)

    def to_local(self, x):
        """The coupled vector in this coupler's working form: a device tensor of the local strips of
        [T | u | v | p] (device mode) or the global NumPy vector."""
        if not self._device:
            return np.array(x, dtype=np.float64)
        if isinstance(x, torch.Tensor):
            return x.to(self.cd._mesh.device, torch.float64).contiguous()
        x = np.asarray(x, dtype=np.float64)
        n, m = self.Ncd, self.Nns
        parts = (x[:n], x[n:n + m], x[n + m:n + 2 * m], x[n + 2 * m:])
        return torch.cat([self.cd._dev(parts[0])] + [self.ns._dev(a) for a in parts[1:]])

    def to_global(self, x):
        """The global NumPy [T | u | v | p] of a working-form vector (gathered across strips)."""
        if not self._device:
            return np.asarray(x, dtype=np.float64)
        T, u, v, p = self._split(x)
        g = lambda s, t: s._out(t, np.zeros(0))  # noqa: E731  (NumPy-like: gathered to the host)
        return np.concatenate((g(self.cd, T), g(self.ns, u), g(self.ns, v), g(self.ns, p)))

    # ------------------------------------------------------------------ component maps
    def _host_call(self, fn, x):
        """Device mode, called with a global NumPy vector (the OpenMDAO-style interface): the same map on the
        working form, the result gathered back."""
        return self.to_global(fn(self.to_local(x)))

    def residuals(self, x):
        """apply_nonlinear of both components (CD :38-39, NS :35-37)."""
        if self._device and not isinstance(x, torch.Tensor):
            return self._host_call(self.residuals, x)
        T, u, v, p = self._split(x)
        t0 = time.perf_counter()
        rT = self.cd._get_residuals(T, self._to_cd(u), self._to_cd(v))
        ru, rv, rp = self.ns._get_residuals(u, v, p, self._to_ns(T))
        self.timing["residuals"] += time.perf_counter() - t0
        self.calls["residuals"] += 1
        return self._join(rT, ru, rv, rp)

    def linearize(self, x):
        """linearize of both components (CD :41-42, NS :39-40); called after residuals(x)."""
        if self._device and not isinstance(x, torch.Tensor):
            x = self.to_local(x)
        T, u, v, _ = self._split(x)
        self.cd._calc_jacobians(T)
        self.ns._calc_jacobians(u, v)

    def jacobian_apply(self, dx):
        """apply_linear, fwd mode (CD :44-49, NS :42-50): the coupled Jacobian on dx."""
        if self._device and not isinstance(dx, torch.Tensor):
            return self._host_call(self.jacobian_apply, dx)
        dT, du, dv, dp = self._split(dx)
        t0 = time.perf_counter()
        rT = self.cd._get_dresiduals(dT, self._to_cd(du), self._to_cd(dv))
        ru, rv, rp = self.ns._get_dresiduals(du, dv, dp, self._to_ns(dT))
        self.timing["jacobian_apply"] += time.perf_counter() - t0
        self.calls["jacobian_apply"] += 1
        return self._join(rT, ru, rv, rp)

    def block_jacobi(self, r):
        """LinearBlockJac(maxiter=1): each component's solve_linear on its own residual block
        (CD :51-57, NS :52-60), zero initial guesses."""
        if self._device and not isinstance(r, torch.Tensor):
            return self._host_call(self.block_jacobi, r)
        rT, ru, rv, rp = self._split(r)
        t0 = time.perf_counter()
        dT = self._timed("cd_update", self.cd._get_update, rT, dT0=self._zeros(self.Ncd, getattr(self, "_ncd_loc", 0)))
        t1 = time.perf_counter()
        z = self._zeros(self.Nns, getattr(self, "_nns_loc", 0))
        du, dv, dp = self._timed("ns_update", self.ns._get_update, ru, rv, rp, du0=z, dv0=z, dp0=z)
        if self.iprint >= 2:
            self._log(f'    block-Jacobi: CD {getattr(self.cd, "matvecs", "?")} matvecs {t1 - t0:.3f} s, '
                      f'NS {getattr(self.ns, "schur_matvecs", "?")} Schur matvecs {time.perf_counter() - t1:.3f} s')
        return self._join(dT, du, dv, dp)

    def gauss_seidel_pass(self, x):
        """One pass of the subsystems' solve_nonlinear in group order (CD :59-61, NS :62-65)."""
        if self._device and not isinstance(x, torch.Tensor):
            return self._host_call(self.gauss_seidel_pass, x)
        T, u, v, p = self._split(x)
        T = self.cd._get_solution(self._to_cd(u), self._to_cd(v), T0=T)
        u, v, p = self.ns._get_solution(self._to_ns(T), u0=u, v0=v, p0=p)
        return self._join(T, u, v, p)

    # ------------------------------------------------------------------ solvers
    def _log(self, msg):
        if self.iprint:
            print(msg, flush=True)

    def solve(self, x0=None, checkpoint=None, resume=False):
        """Run the coupled solve; returns (T, u, v, p) global vectors (NumPy).
        checkpoint(x, k): called after every nonlinear iteration (long runs save their state);
        resume=True: x0 is such a saved state -- continue the Newton iteration without the initial
        subsystem pass."""
        x = self.to_local(np.zeros(self.DOF) if x0 is None else x0)
        self._checkpoint = checkpoint
        x = self._solve_gs(x) if self.mode == 'GS' else self._solve_newton(x, initial_pass=not resume)
        xg = self.to_global(x)
        n, m = self.Ncd, self.Nns
        return xg[:n].copy(), xg[n:n + m].copy(), xg[n + m:n + 2 * m].copy(), xg[n + 2 * m:].copy()

    def _solve_gs(self, x):
        for k in range(self.maxiter):
            x = self.gauss_seidel_pass(x)
            norm = self._norm(self.residuals(x))
            self._log(f'NLBGS {k + 1} ; {norm}')
            self.iterations = k + 1
            if norm <= self.atol_nonlin:
                return x
        raise RuntimeError(f'NLBGS failed to converge in {self.maxiter} iterations')

    def _solve_newton(self, x, initial_pass=True):
        if initial_pass:
            x = self.gauss_seidel_pass(x)  # solve_subsystems=True, max_sub_solves=0: at iteration 0 only
        r = self.residuals(x)
        norm = self._norm(r)
        self._log(f'Newton 0 ; {norm}')
        k = 0
        while norm > self.atol_nonlin:
            if k >= self.maxiter:
                raise RuntimeError(f'Newton failed to converge in {self.maxiter} iterations')
            self.linearize(x)
            if self.mode == 'JNK':
                x = x + self._linear_jnk(-r)
                r = self.residuals(x)
                norm = self._norm(r)
            else:
                x, r, norm = self._armijo_goldstein(x, self.block_jacobi(-r), norm)
            k += 1
            self._log(f'Newton {k} ; {norm}')
            if getattr(self, "_checkpoint", None) is not None:
                self._checkpoint(self.to_global(x), k)
        self.iterations = k
        return x

    # restart-jump safeguard: the block-Jacobi preconditioner is two iterative block solves stopped
    # at mtol_internal sqrt(N); a jump of the preconditioned residual at a GMRES restart (> JUMP_RATIO x the estimate)
    # tightens both block solves' tolerance by JUMP_TIGHTEN for the rest of that linear solve, at most JUMP_MAX times
    JUMP_RATIO, JUMP_TIGHTEN, JUMP_MAX = 10.0, 0.1, 3

    def _tighten_blocks(self, ratio):
        """gmres_left's jump hook: one tightening step of the inner block solves (returns True when applied)."""
        if self._jumps >= self.JUMP_MAX:
            self._log(f'  GMRES restart jump x{ratio:.1f}: block solves already tightened {self._jumps} times')
            return False
        self._jumps += 1
        for s in (self.cd, self.ns):
            if s is not None and hasattr(s, "_mtol"):
                s._mtol *= self.JUMP_TIGHTEN
        self._log(f'  GMRES restart jump x{ratio:.1f}: block solves re-run at {self.JUMP_TIGHTEN ** self._jumps:g} x '
                  f'mtol_internal')
        return True

    def _linear_jnk(self, b):
        """GMRES on the coupled Jacobian, block-Jacobi preconditioned (ScipyKrylov :89-91).  Device mode: the
        Krylov basis and every vector stay on the device (inner products across strips when partitioned).  The
        restart-jump safeguard (_tighten_blocks) leaves a solve whose preconditioner behaves untouched: the same
        arithmetic, the same history."""
        it = [0]

        def cb(presid):
            it[0] += 1
            self._log(f'  GMRES {it[0]} ; {presid}')

        saved = [(s, s._mtol) for s in (self.cd, self.ns) if s is not None and hasattr(s, "_mtol")]
        self._jumps = 0
        try:
            if self._device:
                res = gmres_left(self.jacobian_apply, b, atol=self.atol_gmres, rtol=0.0, restart=self.restart,
                                 maxiter=5000, precond=self.block_jacobi, callback=cb, inner=self._inner,
                                 jump=self._tighten_blocks, jump_ratio=self.JUMP_RATIO)
            else:
                mv = lambda t: torch.from_numpy(self.jacobian_apply(t.numpy()))  # noqa: E731
                pc = lambda t: torch.from_numpy(self.block_jacobi(t.numpy()))  # noqa: E731
                res = gmres_left(mv, torch.from_numpy(np.ascontiguousarray(b)), atol=self.atol_gmres, rtol=0.0,
                                 restart=self.restart, maxiter=5000, precond=pc, callback=cb,
                                 jump=self._tighten_blocks, jump_ratio=self.JUMP_RATIO)
        finally:
            for s, m in saved:
                s._mtol = m
        self.restart_jumps = getattr(self, "restart_jumps", 0) + res.jumps
        if res.info != 0:
            raise RuntimeError(f'GMRES failed to converge in {res.info} restarts')
        return res.x if self._device else res.x.numpy()

    def _armijo_goldstein(self, x, dx, norm0):
        """ArmijoGoldsteinLS(maxiter=AGi, rho=AGr, c=AGc) on the residual norm along dx."""
        alpha = 1.0
        x_new = x + dx
        r_new = self.residuals(x_new)
        n_new = self._norm(r_new)
        for _ in range(self.AGi):
            if n_new <= norm0 * (1.0 - self.AGc * alpha):
                break
            alpha *= self.AGr
            x_new = x + alpha * dx
            r_new = self.residuals(x_new)
            n_new = self._norm(r_new)
        return x_new, r_new, n_new


def run(points_plot, L_x, L_y, Re=1.e3, Ra=1.e3, Pr=0.71, P_cd=4, N_ex_cd=8, N_ey_cd=8, P_ns=4, N_ex_ns=8, N_ey_ns=8,
        mode='JNK', mtol_nonlin=1e-9, AGi=8, AGr=0.8, AGc=0.2, mtol_gmres=1e-10, restart=20, mtol_internal=1e-13):
    """Drop-in for OpenMDAO/Boussinesq_SequentialCoupler.py:10-108 `run` (and the ParallelCoupler's):
    same arguments, returns (T_plot, u_plot, v_plot) interpolated at points_plot."""
    c = BoussinesqCoupler(L_x, L_y, Re, Ra, Pr, P_cd, N_ex_cd, N_ey_cd, P_ns, N_ex_ns, N_ey_ns, mode=mode,
                          mtol_nonlin=mtol_nonlin, AGi=AGi, AGr=AGr, AGc=AGc, mtol_gmres=mtol_gmres, restart=restart,
                          mtol_internal=mtol_internal)
    T, u, v, _ = c.solve()
    return (np.asarray(c.cd._get_interpol(T, points_plot)), np.asarray(c.ns._get_interpol(u, points_plot)),
            np.asarray(c.ns._get_interpol(v, points_plot)))


class ParallelBoussinesqCoupler(BoussinesqCoupler):
    """OpenMDAO/Boussinesq_ParallelCoupler.py:12-121: the coupler's two components in an
    om.ParallelGroup on two ranks -- rank 0 evaluates and solves the convection-diffusion block,
    rank 1 the Navier-Stokes block, concurrently.  Every component map (residuals, linearize,
    Jacobian apply, the block-Jacobi solve of the JNK / NJ preconditioner) runs on its owner rank only
    and the two blocks are reassembled with one all-reduce of the coupled vector (the other rank
    contributes zeros, so the sum is exact) -- torch.distributed: RCCL under "nccl", gloo on the
    host.  The Krylov / Newton iteration on the coupled vector then runs identically on both ranks.

    As in a ParallelGroup, the initial "solve_subsystems" pass (and every GS-mode pass) solves both
    blocks at once from the previous coupling fields (block Jacobi), where the sequential coupler
    uses the new temperature in the NS solve (block Gauss-Seidel)."""

    def __init__(self, *args, dist=None, group=None, **kw):
        super().__init__(*args, **kw)
        self._device = False   # the two blocks meet in a host-side all-reduce of the coupled vector
        if dist is None or dist.get_world_size(group) != 2:
            raise ValueError("the parallel coupler runs on exactly two ranks (CD on rank 0, NS on rank 1)")
        self.dist, self.group = dist, group
        self.rank = dist.get_rank(group)

    def _share(self, part):
        """The coupled vector from this rank's block (rank 0: T block, rank 1: u, v, p blocks)."""
        full = torch.zeros(self.DOF, dtype=torch.float64)
        part = torch.as_tensor(np.asarray(part, dtype=np.float64))
        if self.rank == 0:
            full[:self.Ncd] = part
        else:
            full[self.Ncd:] = part
        dev = None
        if self.dist.get_backend(self.group) == "nccl":   # RCCL reduces device tensors
            dev = torch.device("cuda", torch.cuda.current_device())
            full = full.to(dev)
        self.dist.all_reduce(full, group=self.group)
        return full.cpu().numpy()

    def residuals(self, x):
        T, u, v, p = self._split(x)
        t0 = time.perf_counter()
        if self.rank == 0:
            r = self.cd._get_residuals(T, self._to_cd(u), self._to_cd(v))
        else:
            r = self._join(*self.ns._get_residuals(u, v, p, self._to_ns(T)))
        self.timing["residuals"] += time.perf_counter() - t0
        self.calls["residuals"] += 1
        return self._share(r)

    def linearize(self, x):
        T, u, v, _ = self._split(x)
        if self.rank == 0:
            self.cd._calc_jacobians(T)
        else:
            self.ns._calc_jacobians(u, v)

    def jacobian_apply(self, dx):
        dT, du, dv, dp = self._split(dx)
        t0 = time.perf_counter()
        if self.rank == 0:
            r = self.cd._get_dresiduals(dT, self._to_cd(du), self._to_cd(dv))
        else:
            r = self._join(*self.ns._get_dresiduals(du, dv, dp, self._to_ns(dT)))
        self.timing["jacobian_apply"] += time.perf_counter() - t0
        self.calls["jacobian_apply"] += 1
        return self._share(r)

    def block_jacobi(self, r):
        rT, ru, rv, rp = self._split(r)
        if self.rank == 0:
            d = self._timed("cd_update", self.cd._get_update, rT, dT0=np.zeros(self.Ncd))
        else:
            z = np.zeros(self.Nns)
            d = self._join(*self._timed("ns_update", self.ns._get_update, ru, rv, rp, du0=z, dv0=z, dp0=z))
        return self._share(d)

    def gauss_seidel_pass(self, x):
        T, u, v, p = self._split(x)
        if self.rank == 0:
            d = self.cd._get_solution(self._to_cd(u), self._to_cd(v), T0=T)
        else:
            d = self._join(*self.ns._get_solution(self._to_ns(T), u0=u, v0=v, p0=p))
        return self._share(d)


def run_parallel(points_plot, L_x, L_y, dist, Re=1.e3, Ra=1.e3, Pr=0.71, P_cd=4, N_ex_cd=8, N_ey_cd=8, P_ns=4,
                 N_ex_ns=8, N_ey_ns=8, mode='JNK', mtol_nonlin=1e-9, AGi=8, AGr=0.8, AGc=0.2, mtol_gmres=1e-10,
                 restart=20, mtol_internal=1e-13, group=None):
    """Drop-in for OpenMDAO/Boussinesq_ParallelCoupler.py:12-121 `run`: rank 0 returns
    (T_plot, u_plot, v_plot), rank 1 returns (None, None, None), as the reference's MPI gather does."""
    c = ParallelBoussinesqCoupler(L_x, L_y, Re, Ra, Pr, P_cd, N_ex_cd, N_ey_cd, P_ns, N_ex_ns, N_ey_ns, mode=mode,
                                  mtol_nonlin=mtol_nonlin, AGi=AGi, AGr=AGr, AGc=AGc, mtol_gmres=mtol_gmres,
                                  restart=restart, mtol_internal=mtol_internal, dist=dist, group=group)
    T, u, v, _ = c.solve()
    if dist.get_rank(group) != 0:
        return None, None, None
    return (np.asarray(c.cd._get_interpol(T, points_plot)), np.asarray(c.ns._get_interpol(u, points_plot)),
            np.asarray(c.ns._get_interpol(v, points_plot)))


def partitioned_coupler(dist, L_x, L_y, Re=1.e3, Ra=1.e3, Pr=0.71, P_cd=4, N_ex_cd=8, N_ey_cd=8, P_ns=4, N_ex_ns=8,
                        N_ey_ns=8, group=None, exchange="allreduce", overlap=True, mesh_factory=None,
                        mtol_internal=1e-13, schur_precond="mass", cd_update="distributed", ns_update="distributed",
                        **kw):
    """The element-partitioned Boussinesq coupler (BASELINE cfg5: 128 x 128, P = 12 over 8 GPUs): both
    solvers are strip-partitioned over every rank of `dist` (sem_amd.parallel.Partition -- each rank
    holds the same element-column strip range of the CD and the NS mesh, one GPU per rank), so every
    residual and Jacobian apply is a strip launch plus the RCCL interface exchange, and the Newton updates
    (the block-Jacobi preconditioner's solves) are element-partitioned too (cd_update / ns_update =
    "distributed", the default: strip_solve.StripLineSolver factors each rank's own columns and the ranks
    share a reduced system over the strip-boundary lines; "central" hands a solve to rank 0's whole-mesh
    counterpart).  The coupled Newton-Krylov iteration (OpenMDAO's NewtonSolver + ScipyKrylov on the coupled
    vector, Boussinesq_SequentialCoupler.py:75-93) runs on every rank over its local strips of the coupled
    vector, on the device, with all-reduced inner products.
    Same arguments as BoussinesqCoupler, plus the partition's (group, exchange protocol, overlap,
    mesh_factory for a CPU strip double)."""
    from ..parallel import Partition
    from .convection_diffusion import ConvectionDiffusionSolver
    from .navier_stokes import NavierStokesSolver
    part = lambda: Partition(dist, group=group, exchange=exchange, overlap=overlap, mesh_factory=mesh_factory)  # noqa: E731
    cd = ConvectionDiffusionSolver(L_x=L_x, L_y=L_y, Pe=Re * Pr, P=P_cd, N_ex=N_ex_cd, N_ey=N_ey_cd, T_W=0.5, T_E=-0.5,
                                   mtol=mtol_internal, partition=part(), partition_update=cd_update)
    ns = NavierStokesSolver(L_x=L_x, L_y=L_y, Re=Re, Gr=Ra / Pr, P=P_ns, N_ex=N_ex_ns, N_ey=N_ey_ns, mtol=mtol_internal,
                            mtol_newton=mtol_internal, iprint=[], schur_precond=schur_precond, partition=part(),
                            partition_update=ns_update)
    return BoussinesqCoupler(L_x, L_y, Re, Ra, Pr, P_cd, N_ex_cd, N_ey_cd, P_ns, N_ex_ns, N_ey_ns,
                             mtol_internal=mtol_internal, cd=cd, ns=ns, **kw)
