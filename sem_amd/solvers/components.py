"""OpenMDAO component counterparts: the two implicit components the Boussinesq couplers put in
their coupled group, on the device solver counterparts.

Restates OpenMDAO/ConvectionDiffusion_Component.py:6-61 and OpenMDAO/NavierStokes_Component.py:5-65
(same class names, options, variable names, method signatures, call order and errors), so a
coupler written against OpenMDAO can take these classes unchanged.  OpenMDAO itself is not
installed in this image; when it is importable the components subclass `om.ImplicitComponent`,
otherwise `ImplicitComponent` below, which provides exactly the part of the OpenMDAO component
API the two components use (`options.declare`, `add_input`, `add_output`, `initialize` at
construction).  The vectors OpenMDAO hands in (`inputs`, `outputs`, `residuals`, `d_*`) are
anything with `[name]` access and `in` -- dicts in the tests.

Every method is one or two calls into the solver counterpart (sem_amd.solvers), so each residual /
Jacobian apply is one fused HIP launch and `change_inputs` is the device interpolation kernel.
"""
import numpy as np

try:  # the reference's own framework, when present
    import openmdao.api as _om
    _Base = _om.ImplicitComponent
except ImportError:  # pragma: no cover - the normal case in this image
    _om = None
    _Base = None


class _Options:
    """The subset of OpenMDAO's OptionsDictionary the components use: declare, then set / get."""

    def __init__(self):
        self._decl, self._val = {}, {}

    def declare(self, name, default=None, desc=""):
        self._decl[name] = desc
        if default is not None:
            self._val[name] = default

    def __setitem__(self, name, value):
        if name not in self._decl:
            raise KeyError(f"Option '{name}' cannot be set because it has not been declared.")
        self._val[name] = value

    def __getitem__(self, name):
        if name not in self._decl:
            raise KeyError(f"Option '{name}' cannot be found")
        if name not in self._val:
            raise RuntimeError(f"Option '{name}' is required but has not been set.")
        return self._val[name]

    def __contains__(self, name):
        return name in self._decl


class ImplicitComponent:
    """Stand-in for om.ImplicitComponent (only what the SEM components touch): options are
    declared by initialize() at construction and may be passed as keyword arguments; setup()
    records variables with add_input / add_output (name -> (kind, default value))."""

    def __init__(self, **kwargs):
        self.options = _Options()
        self.variables = {}
        self.initialize()
        for k, v in kwargs.items():
            self.options[k] = v

    def initialize(self):
        pass

    def add_input(self, name, val=1.0, desc=""):
        self.variables[name] = ("input", np.array(val, dtype=np.float64))

    def add_output(self, name, val=1.0, desc=""):
        self.variables[name] = ("output", np.array(val, dtype=np.float64))


if _Base is None:
    _Base = ImplicitComponent


def transfer(field, src, dst):
    """A field of solver `src` evaluated at the nodes of solver `dst` -- the change_inputs map of
    both components (ConvectionDiffusion_Component.py:23-36, NavierStokes_Component.py:22-33).
    dst._get_vector hands its node coordinates as two flat arrays; src._get_interpol takes a mesh
    grid, so the coordinates are reshaped to dst's (2, P N_ex + 1, P N_ey + 1) grid and the result
    flattened back.  Linear in `field`; applied even when the two meshes coincide, as there."""
    grid = (2, dst._P * dst._N_ex + 1, dst._P * dst._N_ey + 1)
    return dst._get_vector(
        f_func=lambda x, y: np.asarray(src._get_interpol(field, np.reshape((x, y), grid))).flatten())


def _fwd_only(mode):
    if mode != 'fwd':
        raise ValueError('only forward mode implemented')


class ConvectionDiffusion_Component(_Base):
    """OpenMDAO/ConvectionDiffusion_Component.py:6-61: output T_cd, inputs u_ns, v_ns."""

    def initialize(self):
        self.options.declare('solver_CD', desc='convection-diffusion solver object')
        self.options.declare('solver_NS', desc='NAVIER-STOKES solver object')

    def setup(self):
        self.cd, self.ns = self.options['solver_CD'], self.options['solver_NS']
        self.add_output('T_cd', val=np.zeros(self.cd.N), desc='T as CD global vector')
        self.add_input('u_ns', val=np.zeros(self.ns.N), desc='u as NS global vector')
        self.add_input('v_ns', val=np.zeros(self.ns.N), desc='v as NS global vector')
        self.iter_count_solve = 0  # number of _get_update calls

    def change_inputs(self, u_ns, v_ns):
        """(:23-36) the NS velocity at the CD nodes."""
        return transfer(u_ns, self.ns, self.cd), transfer(v_ns, self.ns, self.cd)

    def apply_nonlinear(self, inputs, outputs, residuals, *args):
        """(:38-39)"""
        residuals['T_cd'] = self.cd._get_residuals(outputs['T_cd'], *self.change_inputs(inputs['u_ns'],
                                                                                       inputs['v_ns']))

    def linearize(self, inputs, outputs, partials, *args):
        """(:41-42)"""
        self.cd._calc_jacobians(outputs['T_cd'])

    def apply_linear(self, inputs, outputs, d_inputs, d_outputs, d_residuals, mode, *args):
        """(:44-49) forward mode only; an absent d_outputs['T_cd'] counts as zero."""
        _fwd_only(mode)
        dT = d_outputs['T_cd'] if 'T_cd' in d_outputs else np.zeros(self.cd.N)
        d_residuals['T_cd'] = self.cd._get_dresiduals(dT, *self.change_inputs(d_inputs['u_ns'], d_inputs['v_ns']))

    def solve_linear(self, d_outputs, d_residuals, mode):
        """(:51-57) one Newton update from the current d_outputs as initial guess."""
        _fwd_only(mode)
        d_outputs['T_cd'] = self.cd._get_update(d_residuals['T_cd'], dT0=d_outputs['T_cd'])
        self.iter_count_solve += 1

    def solve_nonlinear(self, inputs, outputs):
        """(:59-61) the CD problem is linear in T: one update."""
        outputs['T_cd'] = self.cd._get_solution(*self.change_inputs(inputs['u_ns'], inputs['v_ns']),
                                                T0=outputs['T_cd'])
        self.iter_count_solve += 1


class NavierStokes_Component(_Base):
    """OpenMDAO/NavierStokes_Component.py:5-65: outputs u_ns, v_ns, p_ns, input T_cd."""

    _OUT = ('u_ns', 'v_ns', 'p_ns')

    def initialize(self):
        self.options.declare('solver_NS', desc='NAVIER-STOKES solver object')
        self.options.declare('solver_CD', desc='convection-diffusion solver object')

    def setup(self):
        self.ns, self.cd = self.options['solver_NS'], self.options['solver_CD']
        self.add_input('T_cd', val=np.zeros(self.cd.N), desc='T as CD global vector')
        for name, what in zip(self._OUT, 'uvp'):
            self.add_output(name, val=np.zeros(self.ns.N), desc=f'{what} as NS global vector')
        self.iter_count_solve = 0  # number of _get_update calls

    def change_inputs(self, T_cd):
        """(:22-33) the CD temperature at the NS nodes."""
        return transfer(T_cd, self.cd, self.ns)

    def _store(self, vec, values):
        for name, a in zip(self._OUT, values):
            vec[name] = a

    def apply_nonlinear(self, inputs, outputs, residuals, *args):
        """(:35-37)"""
        self._store(residuals, self.ns._get_residuals(*(outputs[n] for n in self._OUT),
                                                      self.change_inputs(inputs['T_cd'])))

    def linearize(self, inputs, outputs, partials, *args):
        """(:39-40)"""
        self.ns._calc_jacobians(outputs['u_ns'], outputs['v_ns'])

    def apply_linear(self, inputs, outputs, d_inputs, d_outputs, d_residuals, mode, *args):
        """(:42-50) forward mode only; absent d_outputs entries count as zero."""
        _fwd_only(mode)
        d = [d_outputs[n] if n in d_outputs else np.zeros(self.ns.N) for n in self._OUT]
        self._store(d_residuals, self.ns._get_dresiduals(*d, self.change_inputs(d_inputs['T_cd'])))

    def solve_linear(self, d_outputs, d_residuals, mode):
        """(:52-60) the velocity-pressure update, current d_outputs as initial guesses."""
        _fwd_only(mode)
        self._store(d_outputs, self.ns._get_update(*(d_residuals[n] for n in self._OUT),
                                                   du0=d_outputs['u_ns'], dv0=d_outputs['v_ns'],
                                                   dp0=d_outputs['p_ns']))
        self.iter_count_solve += 1

    def solve_nonlinear(self, inputs, outputs):
        """(:62-65) the inner Newton iteration; counts its _get_update calls (ns._k)."""
        self._store(outputs, self.ns._get_solution(self.change_inputs(inputs['T_cd']), u0=outputs['u_ns'],
                                                   v0=outputs['v_ns'], p0=outputs['p_ns']))
        self.iter_count_solve += self.ns._k
