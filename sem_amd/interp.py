"""Element interpolation / grid transfer on the GPU (SEM.py:248-273).

Host side only decides, per plot row / column, which element holds it and its
reference coordinate (SEM.x2xi, SEM.py:23-36) and builds the (P+1)-wide
Lagrange evaluation rows; the contraction with the element coefficients runs in
libsemops (sem_eval_interpolation).
"""
import ctypes as C

import numpy as np
import torch

from . import GLL, _lib
from .device import get_mesh


def eval_interpolation(u_e, points_e, points_plot):
    from .SEM import x2xi
    nex, ney, P = u_e.shape[0], u_e.shape[1], u_e.shape[2] - 1
    x_e = points_e[0, :, 0, :, 0]
    y_e = points_e[1, 0, :, 0, :]
    dx = x_e[0, -1] - x_e[0, 0]
    dy = y_e[0, -1] - y_e[0, 0]
    m_plot, xi_plot = x2xi(points_plot[0][:, 0], dx)
    n_plot, eta_plot = x2xi(points_plot[1][0, :], dy)
    mesh = get_mesh(P, nex, ney, 1.0, 1.0)
    dev = mesh.device
    Sx = GLL.standard_evaluation_matrix(P, np.clip(xi_plot, -1, 1))
    Sy = GLL.standard_evaluation_matrix(P, np.clip(eta_plot, -1, 1))
    # points outside [0, L] get index -1 and stay 0, as the reference leaves them
    mi = np.where((m_plot >= 0) & (m_plot < nex), m_plot, -1).astype(np.int32)
    ni = np.where((n_plot >= 0) & (n_plot < ney), n_plot, -1).astype(np.int32)
    on_dev = isinstance(u_e, torch.Tensor)
    ue = mesh.to_device(u_e)
    t = [torch.as_tensor(a, device=dev) for a in (mi, Sx, ni, Sy)]
    na, nb = mi.size, ni.size
    out = torch.zeros(na * nb, dtype=torch.float64, device=dev)
    p = lambda a: C.c_void_p(a.data_ptr())  # noqa: E731
    _lib.check(_lib.load().sem_eval_interpolation(mesh._h, p(ue), na, p(t[0]), p(t[1]), nb, p(t[2]), p(t[3]), p(out),
                                                   mesh.stream_ptr()))
    out = out.reshape(na, nb)
    return out if on_dev else out.cpu().numpy()
