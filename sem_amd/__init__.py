"""sem_amd -- MI355X-native spectral-element operator layer.

Drop-in for the hot path of Tangxiaotian11/SEM (Solvers/GLL.py + Solvers/SEM.py):

    from sem_amd import GLL, SEM
    K = SEM.global_stiffness_matrix(P, N_ex, N_ey, dx, dy)   # matrix-free, on the GPU
    y = K @ T

The arithmetic runs in hand-written HIP kernels for gfx950 (sem_amd/csrc,
C ABI in include/sem_ops.h); PyTorch-ROCm supplies device memory, streams and
torch.distributed (RCCL) for the element-strip partition.
"""
from . import GLL, SEM  # noqa: F401

__all__ = ["GLL", "SEM"]
