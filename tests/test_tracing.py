"""CPU tests of sem_amd/tracing.py, the phase timer behind tools/strip_profile.py: phases are free when no trace
is active, nest (a parent includes its children), count calls per name, and split per unit; the device GMRES
reports its matvec / orthogonalisation phases through it."""
import time

import numpy as np
import torch

from sem_amd import tracing
from sem_amd.krylov import gmres


def test_phases_off_by_default():
    with tracing.phase("x"):
        pass
    assert tracing.begin("y") is None
    tracing.end(None)
    tracing.count("z")            # no active trace: nothing to record, nothing raised


def test_phases_nest_and_count():
    tr = tracing.Trace(device="cpu")
    with tracing.tracing(tr):
        for _ in range(3):
            with tracing.phase("outer"):
                time.sleep(0.002)
                with tracing.phase("inner"):
                    time.sleep(0.001)
        tok = tracing.begin("span")
        tracing.end(tok)
        tracing.count("collectives", 2)
    assert tracing._ACTIVE is None
    rows = {name: (calls, dev, host) for name, calls, dev, host in tr.table(per=3)}
    assert rows["outer"][0] == 1.0 and rows["inner"][0] == 1.0 and rows["span"][0] == 1 / 3
    assert rows["outer"][2] >= rows["inner"][2] >= 0.9          # host ms per unit; the parent includes the child
    assert rows["outer"][1] == 0.0                              # no device on the CPU
    assert tr.counters == {"collectives": 2}
    tr.reset()
    assert tr.stats == {} and tr.counters == {}


def test_gmres_reports_its_phases():
    r = np.random.default_rng(3)
    A = torch.as_tensor(np.eye(40) * 4 + r.uniform(-1, 1, (40, 40)))
    b = torch.as_tensor(r.uniform(-1, 1, 40))
    tr = tracing.Trace(device="cpu")
    with tracing.tracing(tr):
        res = gmres(lambda x: A @ x, b, atol=1e-12)
    stats = tr.resolve()
    # one traced matvec per Arnoldi step; the true-residual check after a cycle is the caller's matvec, untraced
    assert stats["krylov.matvec"][0] == stats["krylov.orthogonalise"][0] == res.iters <= res.matvecs
