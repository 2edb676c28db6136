"""Per-launch HIP-event tracing of the hot kernels (used by bench.py for the roofline).

When active, every conv launch records a start/end torch.cuda.Event on the stream it is
launched on, with its kernel instantiation name and algorithmic FLOPs / bytes; after a
synchronize the records give per-kernel average duration and achieved TFLOP/s or GB/s,
directly comparable with ``rocprofv3 --kernel-trace --stats`` averages for the same names.
"""
import contextlib

import torch

_STATE = {'active': False, 'records': [], 'pool': []}


def start():
    _STATE['active'] = True
    _STATE['records'] = []


def stop():
    _STATE['active'] = False
    torch.cuda.synchronize()
    recs = _STATE['records']
    _STATE['records'] = []
    out = {}
    for name, flops, nbytes, s, e in recs:
        d = out.setdefault(name, {'count': 0, 'ms': 0.0, 'flops': 0.0, 'bytes': 0.0})
        d['count'] += 1
        d['ms'] += s.elapsed_time(e)
        d['flops'] += flops
        d['bytes'] += nbytes
        _STATE['pool'].extend((s, e))
    return out


def _event():
    pool = _STATE['pool']
    return pool.pop() if pool else torch.cuda.Event(enable_timing=True)


@contextlib.contextmanager
def span(name, flops=0.0, nbytes=0.0):
    if not _STATE['active']:
        yield
        return
    s, e = _event(), _event()
    s.record()
    yield
    e.record()
    _STATE['records'].append((name, float(flops), float(nbytes), s, e))
