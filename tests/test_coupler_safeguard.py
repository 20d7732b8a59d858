"""The Boussinesq coupler's restart-jump safeguard (sem_amd/solvers/boussinesq.py) on CPU: the
block-Jacobi preconditioner of the coupled JNK iteration is a pair of iterative block solves stopped at mtol_internal;
a jump of the preconditioned residual at a GMRES restart tightens both block solves for the rest of that linear
solve, and their tolerances are restored afterwards (OpenMDAO/Boussinesq_SequentialCoupler.py:80-89 runs the same
ScipyKrylov / LinearBlockJac structure)."""
import types

import numpy as np
import torch

from sem_amd.solvers.boussinesq import BoussinesqCoupler


class _Block:
    """A stand-in block solver: its solve is exact up to a perturbation proportional to its _mtol."""

    def __init__(self, mtol, seed):
        self._mtol = mtol
        self.rng = np.random.default_rng(seed)
        self.seen = []


def _coupler(A, d, mtol):
    c = types.SimpleNamespace()
    c.cd, c.ns = _Block(mtol, 1), _Block(mtol, 2)
    c._device, c.restart, c.atol_gmres, c._inner, c.iprint = False, 10, 1e-9, None, 0
    c.JUMP_RATIO, c.JUMP_TIGHTEN, c.JUMP_MAX = BoussinesqCoupler.JUMP_RATIO, 0.1, 3
    c._log = lambda m: None
    c.jacobian_apply = lambda x: A @ x
    n = A.shape[0] // 2

    def block_jacobi(r):
        z = r / d
        for blk, sl in ((c.cd, slice(0, n)), (c.ns, slice(n, None))):
            blk.seen.append(blk._mtol)
            z[sl] += blk._mtol * np.linalg.norm(z[sl]) / np.sqrt(n) * blk.rng.uniform(-1, 1, z[sl].shape)
        return z
    c.block_jacobi = block_jacobi
    c._tighten_blocks = types.MethodType(BoussinesqCoupler._tighten_blocks, c)
    return c


def test_restart_jump_tightens_the_block_solves_and_restores_them():
    r = np.random.default_rng(7)
    n = 300
    A = np.diag(np.linspace(1.0, 50.0, n)) + 0.3 * r.standard_normal((n, n)) / np.sqrt(n)
    b = r.standard_normal(n)
    d = np.diag(A).copy()
    c = _coupler(A, d, 1e-2)
    x = BoussinesqCoupler._linear_jnk(c, b)
    assert np.linalg.norm(A @ x - b) <= c.atol_gmres
    assert c.restart_jumps >= 1 and c._jumps >= 1
    assert min(c.ns.seen) < 1e-2 and min(c.cd.seen) < 1e-2     # the block solves ran tighter after the jump
    assert c.cd._mtol == 1e-2 and c.ns._mtol == 1e-2            # and the tolerances are back afterwards
    # consistent blocks: no jump, no tightening
    c0 = _coupler(A, d, 0.0)
    BoussinesqCoupler._linear_jnk(c0, b)
    assert c0.restart_jumps == 0 and set(c0.ns.seen) == {0.0}


def test_tightening_is_capped():
    c = types.SimpleNamespace(cd=_Block(1e-13, 1), ns=_Block(1e-13, 2), _jumps=0, JUMP_MAX=2, JUMP_TIGHTEN=0.1,
                              _log=lambda m: None)
    f = types.MethodType(BoussinesqCoupler._tighten_blocks, c)
    assert f(20.0) and f(20.0) and not f(20.0)
    assert abs(c.ns._mtol - 1e-15) < 1e-27 and c._jumps == 2
