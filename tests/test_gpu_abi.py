"""GPU tests of the C-ABI guards: launchers run only on their handle's device, the HIP Krylov
sweeps refuse non-float64 operands, and the kernel-selection knobs never change a result."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _poke_device(mesh, dev):
    """Overwrite the device field of the opaque handle (struct sem_handle, sem_internal.h:
    int P, nex, ney, ex_begin, ex_end, device) -- the only way to make a handle's device differ
    from the current one on a one-GPU box."""
    p = C.cast(mesh._h, C.POINTER(C.c_int))
    old = p[5]
    p[5] = dev
    return old


def test_launchers_refuse_a_handle_of_another_device(gpu):
    from sem_amd import _lib
    from sem_amd.device import Mesh
    mesh = Mesh(4, 3, 3, 1 / 3, 1 / 3, device=0)
    x = mesh.to_device(np.ones(mesh.n_local))
    y0 = mesh.apply(x, c_stiff=1.0)
    if torch.cuda.device_count() > 1:   # the real situation: another device is current
        with torch.cuda.device(1):
            with pytest.raises(ValueError, match="device"):
                mesh.apply(x, c_stiff=1.0)
    old = _poke_device(mesh, 7)
    try:
        with pytest.raises(ValueError, match="belongs to device 7"):
            mesh.apply(x, c_stiff=1.0)
        with pytest.raises(ValueError, match="device"):
            mesh.gather_elements(x)
        with pytest.raises(ValueError, match="device"):
            mesh.dss(torch.zeros((3, 3, 5, 5), dtype=torch.float64, device=mesh.device))
    finally:
        _poke_device(mesh, old)
    assert torch.equal(mesh.apply(x, c_stiff=1.0), y0)
    assert _lib.SEM_EINVAL == 1


def test_sweeps_refuse_other_dtypes(gpu):
    from sem_amd.krylov import _DeviceSweeps, gmres
    V = torch.zeros((4, 100), dtype=torch.float32, device=gpu)
    with pytest.raises(ValueError):
        _DeviceSweeps(V)
    Vd = torch.randn((4, 100), dtype=torch.float64, device=gpu)
    s = _DeviceSweeps(Vd)
    with pytest.raises(ValueError):
        s.dot2(2, torch.ones(100, dtype=torch.float32, device=gpu), Vd[0])
    with pytest.raises(ValueError):
        s.update(2, torch.ones(4, dtype=torch.float64, device=gpu), torch.ones(50, dtype=torch.float64, device=gpu))
    # float32 systems take torch's GEMV route and still solve
    A = torch.eye(50, dtype=torch.float32, device=gpu) * 2 + 0.01 * torch.randn(50, 50, device=gpu)
    b = torch.ones(50, dtype=torch.float32, device=gpu)
    r = gmres(lambda v: A @ v, b, atol=1e-4, restart=50)
    assert r.info == 0 and torch.linalg.vector_norm(A @ r.x - b).item() < 1e-3


def test_tuning_knobs_do_not_change_results(gpu, tuning):
    """Every band-kernel knob value selects a variant with bitwise-identical results; retired knobs are refused."""
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    mesh = get_mesh(8, 20, 17, 1 / 20, 1 / 17)
    r = np.random.default_rng(3)
    X, U, V = (mesh.to_device(r.uniform(-1, 1, mesh.n_local)) for _ in range(3))
    kw = dict(c_stiff=1.0, c_gradx=40.0, cu=U, c_grady=40.0, cv=V, dir_mode=_lib.DIR_IDENTITY,
              dir_sides=_lib.SIDE_W | _lib.SIDE_E)
    base = mesh.apply(X, **kw)
    for knob, vals in ((_lib.TUNE_BAND_KP, (-1, 0)), (_lib.TUNE_BAND_TILE, (3, 4))):
        for v in vals:
            tuning(knob, v)
            assert torch.equal(mesh.apply(X, **kw), base), (knob, v)
        tuning(knob, 0)
