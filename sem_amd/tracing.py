"""Per-phase timing of the solver paths: HIP events on the launch stream (device time) beside host wall time.

The reference times only its LU (`time.perf_counter`, NavierStokes_Solver.py:177,186-187) and prints
iteration counts.  Here the element-partitioned Schur matvec and the Krylov step are split
into named phases (`with phase("name"):`) that cost one attribute test when tracing is off.  With a
`Trace` active (tools/strip_profile.py), every phase records a HIP event pair on the current stream and,
when `sync` is set, synchronises at its end, so the phase's host wall time includes everything the host
waited for in it (gloo's host-staged collectives, `.item()`).  Phases nest; a parent includes its
children.  Tracing is refused inside a stream capture (an event pair there would be captured, not timed).
"""
import contextlib
import time

import torch

_ACTIVE = None


class Trace:
    """Collects phases: name -> [calls, device seconds, host seconds]."""

    def __init__(self, device=None, sync=True):
        self.device = torch.device(device) if device is not None else None
        self.sync = sync
        self.pending = []            # (name, e0, e1, host seconds) until resolve()
        self.stats = {}
        self.counters = {}

    def count(self, key, n=1):
        self.counters[key] = self.counters.get(key, 0) + n

    def resolve(self):
        """Turn the recorded event pairs into device times (synchronises)."""
        if self.pending and self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        for name, e0, e1, host in self.pending:
            s = self.stats.setdefault(name, [0, 0.0, 0.0])
            s[0] += 1
            s[1] += e0.elapsed_time(e1) / 1e3 if e0 is not None else 0.0
            s[2] += host
        self.pending.clear()
        return self.stats

    def reset(self):
        self.resolve()
        self.stats.clear()
        self.counters.clear()

    def table(self, per=1):
        """Rows (name, calls, device ms, host ms) per `per` units (e.g. per matvec)."""
        self.resolve()
        return [(k, v[0] / per, 1e3 * v[1] / per, 1e3 * v[2] / per) for k, v in sorted(self.stats.items())]


@contextlib.contextmanager
def tracing(trace):
    """Activate `trace` for the enclosed code."""
    global _ACTIVE
    prev, _ACTIVE = _ACTIVE, trace
    try:
        yield trace
    finally:
        _ACTIVE = prev


@contextlib.contextmanager
def phase(name):
    tr = _ACTIVE
    if tr is None:
        yield
        return
    cuda = tr.device is not None and tr.device.type == "cuda"
    if cuda and torch.cuda.is_current_stream_capturing():
        yield
        return
    e0 = e1 = None
    if cuda:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if cuda:
            e1.record()
            if tr.sync:
                torch.cuda.synchronize(tr.device)
        tr.pending.append((name, e0, e1, time.perf_counter() - t0))


def begin(name):
    """phase() as a begin / end pair for spans that do not fit one block: returns a token for end()."""
    if _ACTIVE is None:
        return None
    cm = phase(name)
    cm.__enter__()
    return cm


def end(token):
    if token is not None:
        token.__exit__(None, None, None)


def count(key, n=1):
    if _ACTIVE is not None:
        _ACTIVE.count(key, n)
