"""Element-strip partition on ONE GPU: every strip is its own handle; the interface
exchange (pack -> sum over strips -> unpack) is emulated by summing the packed buffers,
which is exactly what the RCCL all-reduce computes.  The assembled strips must equal
the unpartitioned apply (including Dirichlet rows on interface lines)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-300)


@pytest.mark.parametrize("algo", [1, 2, 3, 4])
@pytest.mark.parametrize("P,nex,ney,G", [(4, 6, 5, 2), (8, 9, 7, 3), (8, 64, 64, 8), (12, 5, 4, 5), (16, 4, 3, 2)])
def test_strip_partition_matches_full_apply(gpu, P, nex, ney, G, algo):
    from sem_amd import _lib
    from sem_amd.device import get_mesh
    from sem_amd.parallel import StripPartition
    dx, dy = 1.0 / nex, 1.0 / ney
    full = get_mesh(P, nex, ney, dx, dy)
    N = full.n_local
    gen = torch.Generator(device=full.device).manual_seed(P * 100 + G)
    x, u, v, g = (torch.rand(N, dtype=torch.float64, device=full.device, generator=gen) * 2 - 1 for _ in range(4))
    kw = dict(c_mass=0.3, c_stiff=1.0, c_gradx=40.0, c_grady=40.0, dir_mode=_lib.DIR_IDENTITY,
              dir_sides=_lib.SIDE_W | _lib.SIDE_E | _lib.SIDE_S, algo=algo)
    want = full.apply(x, cu=u, cv=v, dir_val=g, **kw)
    part = StripPartition(nex, G)
    bufs, outs, meshes = [], [], []
    for r in range(G):
        eb, ee = part.local_range(r)
        m = get_mesh(P, nex, ney, dx, dy, eb, ee)
        sl = slice(m.dof_begin, m.dof_begin + m.n_local)
        y = m.apply(x[sl].contiguous(), cu=u[sl].contiguous(), cv=v[sl].contiguous(), dir_val=g[sl].contiguous(),
                    **kw)
        buf = torch.empty((G - 1) * m.NY, dtype=torch.float64, device=m.device)
        m.interface_pack(y, part.bounds, buf)
        bufs.append(buf)
        outs.append((m, sl, y))
    total = torch.stack(bufs).sum(0)  # what the all-reduce returns on every rank
    for m, sl, y in outs:
        m.interface_unpack(total, part.bounds, y)
        assert rel(y, want[sl]) < 1e-13
