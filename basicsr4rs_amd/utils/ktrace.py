"""Per-launch HIP-event tracing of the hot kernels (used by bench.py for the roofline).

When active, every conv launch records a start/end torch.cuda.Event on the stream it is
launched on, with its kernel instantiation name and algorithmic FLOPs / bytes; after a
synchronize the records give per-kernel average duration and achieved TFLOP/s or GB/s,
directly comparable with ``rocprofv3 --kernel-trace --stats`` averages for the same names.

A span may also carry a ``relaunch`` closure that re-issues exactly that launch (same
arguments, buffers kept alive by the closure).  ``time_relaunch(name)`` replays every launch
of a kernel name recorded by the last trace back to back between two events -- the kernel's
steady-state average duration without per-launch event packets in between, which is what
rocprofv3 reports for the same kernel inside the timed graph replays.
"""
import contextlib

import torch

_STATE = {'active': False, 'records': [], 'pool': [], 'relaunch': {}}


def active():
    return _STATE['active']


def start():
    _STATE['active'] = True
    _STATE['records'] = []
    _STATE['relaunch'] = {}


def stop():
    _STATE['active'] = False
    torch.cuda.synchronize()
    recs = _STATE['records']
    _STATE['records'] = []
    out = {}
    for name, flops, nbytes, launches, s, e in recs:
        d = out.setdefault(name, {'count': 0, 'launches': 0, 'ms': 0.0, 'flops': 0.0, 'bytes': 0.0})
        d['count'] += 1
        d['launches'] += launches
        d['ms'] += s.elapsed_time(e)
        d['flops'] += flops
        d['bytes'] += nbytes
        _STATE['pool'].extend((s, e))
    return out


def _event():
    pool = _STATE['pool']
    return pool.pop() if pool else torch.cuda.Event(enable_timing=True)


class _Span:
    """Event pair around one traced launch (see ``span``)."""
    __slots__ = ('name', 'flops', 'nbytes', 'relaunch', 'launches', 's', 'e')

    def __init__(self, name, flops, nbytes, relaunch, launches):
        self.name, self.flops, self.nbytes, self.relaunch, self.launches = name, flops, nbytes, relaunch, launches

    def __enter__(self):
        self.s, self.e = _event(), _event()
        self.s.record()
        return self

    def __exit__(self, exc_type, *exc):
        self.e.record()
        if exc_type is None:
            _STATE['records'].append((self.name, float(self.flops), float(self.nbytes), int(self.launches), self.s, self.e))
            if self.relaunch is not None:
                _STATE['relaunch'].setdefault(self.name, []).append(self.relaunch)
        return False


_NULL = contextlib.nullcontext()


def span(name, flops=0.0, nbytes=0.0, relaunch=None, launches=1):
    """One op call of kernel ``name``: its algorithmic FLOPs and HBM bytes (every operand the call
    reads or writes, once) and the number of kernel launches it makes (``launches``: the per-launch
    unit of rocprof's --stats, e.g. the 64-channel slices of a sliced band conv).  Outside a trace
    a shared no-op context (every train step enters ~1 k of these on the host)."""
    if not _STATE['active']:
        return _NULL
    return _Span(name, flops, nbytes, relaunch, launches)


def relaunch_count(name):
    return len(_STATE['relaunch'].get(name, ()))


def time_relaunch(name, reps=3):
    """Average ms per launch of ``name`` re-issued back to back (all launches of the last trace,
    ``reps`` passes after one warm-up pass), or None when its launches carry no closure."""
    fns = _STATE['relaunch'].get(name)
    if not fns:
        return None
    for f in fns:
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        for f in fns:
            f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * len(fns))


def clear_relaunch():
    _STATE['relaunch'] = {}
