import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP kernels through the C ABI")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    return torch.device("cuda", 0)


@pytest.fixture
def tuning():
    """set(knob, value): change a libsemops kernel-selection knob (include/sem_ops.h enum sem_tune)
    for one test; the previous values are restored afterwards."""
    import ctypes as C

    from sem_amd import _lib
    lib = _lib.load()
    saved = {}

    def set_(knob, value):
        if knob not in saved:
            v = C.c_int()
            _lib.check(lib.sem_get_tuning(knob, C.byref(v)))
            saved[knob] = v.value
        _lib.check(lib.sem_set_tuning(knob, int(value)))

    yield set_
    for k, v in saved.items():
        lib.sem_set_tuning(k, v)
