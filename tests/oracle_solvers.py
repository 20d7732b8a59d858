"""Test helper (not a test module): the reference solvers' private-method interface
(ConvectionDiffusion_Solver.py / NavierStokes_Solver.py, as the OpenMDAO components call it) on top
of the CPU oracle, so the coupler logic can run where no GPU exists (gloo tests)."""
import numpy as np
import scipy.sparse.linalg as spla

from oracle import sem_oracle as O


class _Nodal:
    """_get_vector / _get_interpol (ConvectionDiffusion_Solver.py:172-190; the NS solver's are the
    same): what the OpenMDAO components' change_inputs calls."""

    def _nodal(self, L_x, L_y, P, N_ex, N_ey):
        self._P, self._N_ex, self._N_ey = P, N_ex, N_ey
        self.points_e = O.element_nodes(P, N_ex, N_ey, L_x / N_ex, L_y / N_ey)

    def _get_vector(self, f_func):
        return f_func(self.points[0], self.points[1])

    def _get_interpol(self, f, points_plot):
        f_e = O.scatter(np.asarray(f), self._P, self._N_ex, self._N_ey)
        return O.eval_interpolation(f_e, self.points_e, points_plot)


class OracleCD(_Nodal):
    def __init__(self, L_x, L_y, Pe, P, N_ex, N_ey, T_W=None, T_E=None, mtol=1e-7):
        self.o = O.CDOracle(L_x, L_y, Pe, P, N_ex, N_ey, T_W=T_W, T_E=T_E)
        self.N, self.points = self.o.N, self.o.points
        self._nodal(L_x, L_y, P, N_ex, N_ey)
        self._mtol = mtol

    def _get_residuals(self, T, u, v):
        return self.o.residuals(np.asarray(T), np.asarray(u), np.asarray(v))

    def _calc_jacobians(self, T):
        self.o.calc_jacobians(np.asarray(T))

    def _get_dresiduals(self, dT, du=None, dv=None):
        return self.o.dresiduals(np.asarray(dT), du, dv)

    def _get_update(self, dres, dT0=None):
        A = spla.LinearOperator((self.N,) * 2, matvec=lambda d: self.o.dresiduals(np.ravel(d)), dtype=float)
        dT, info = spla.lgmres(A, np.asarray(dres), x0=dT0, atol=self._mtol * np.sqrt(self.N), rtol=0,
                               inner_m=int(self.N * 0.3))
        assert info == 0
        return dT

    def _get_solution(self, u, v, T0=None):
        T = np.zeros(self.N) if T0 is None else np.asarray(T0)
        return T + self._get_update(-self._get_residuals(T, u, v))


class OracleNS(_Nodal):
    def __init__(self, L_x, L_y, Re, Gr, P, N_ex, N_ey, mtol=1e-7, mtol_newton=1e-5):
        self.o = O.NSOracle(L_x, L_y, Re, Gr, P, N_ex, N_ey)
        self.N, self.points = self.o.N, self.o.points
        self._nodal(L_x, L_y, P, N_ex, N_ey)
        self._mtol, self._mtol_newton = mtol, mtol_newton

    def _get_residuals(self, u, v, p, T):
        return self.o.residuals(np.asarray(u), np.asarray(v), np.asarray(p), np.asarray(T))

    def _calc_jacobians(self, u, v):
        self.o.calc_jacobians(np.asarray(u), np.asarray(v))

    def _get_dresiduals(self, du, dv, dp, dT=None):
        return self.o.dresiduals(np.asarray(du), np.asarray(dv), np.asarray(dp), dT)

    def _get_update(self, ru, rv, rc, du0=None, dv0=None, dp0=None):
        return self.o.update(np.asarray(ru), np.asarray(rv), np.asarray(rc), mtol=self._mtol, dp0=dp0)[:3]

    def _get_solution(self, T, u0=None, v0=None, p0=None):
        u, v, p, hist = self.o.solution(np.asarray(T), mtol=self._mtol, mtol_newton=self._mtol_newton, u0=u0,
                                        v0=v0, p0=p0)
        self._k = len(hist) - 1   # Newton updates taken (NavierStokes_Solver.py:241-270)
        return u, v, p
