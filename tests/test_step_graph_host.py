"""SegmentedStepGraph's capture bookkeeping on the host (no GPU: the CUDA graph / stream API is
replaced by recording fakes).  ADVICE r3: an exception raised inside ``capture`` (e.g. the
reducer's extra-contribution RuntimeError) must end the open segment's capture before it
propagates, so the capture stream is not left in capture mode."""
import contextlib

import pytest
import torch

from basicsr4rs_amd.utils import step_graph


class _FakeGraph:
    log = []
    modes = []

    def capture_begin(self, pool=None, capture_error_mode="global"):
        _FakeGraph.modes.append(capture_error_mode)
        _FakeGraph.log.append('begin')

    def capture_end(self):
        _FakeGraph.log.append('end')


class _FakeStream:

    def wait_stream(self, other):
        pass


class _FakeReducer:

    def __init__(self):
        self.on_issue = None
        self.issue_log = []
        self.resets = 0

    def flush(self):
        pass

    def reset(self):
        self.resets += 1


@pytest.fixture
def fake_cuda(monkeypatch):
    _FakeGraph.log = []
    monkeypatch.setattr(torch.cuda, 'CUDAGraph', _FakeGraph)
    monkeypatch.setattr(torch.cuda, 'Stream', lambda *a, **k: _FakeStream())
    monkeypatch.setattr(torch.cuda, 'stream', lambda s: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, 'graph_pool_handle', lambda: None)
    monkeypatch.setattr(torch.cuda, 'synchronize', lambda *a: None)
    monkeypatch.setattr(torch.cuda, 'current_stream', lambda *a: _FakeStream())
    return _FakeGraph


def test_exception_mid_capture_ends_open_segment(fake_cuda):
    red = _FakeReducer()
    seg = step_graph.SegmentedStepGraph(red, 'cpu')

    def body(before_backward):
        seg.cut(0)  # one completed backward segment, the next one open
        raise RuntimeError('injected mid-capture failure')

    with pytest.raises(RuntimeError, match='injected'):
        seg.capture(body, lambda: None)
    # every begun capture was ended, nothing half-captured is kept
    assert fake_cuda.log.count('begin') == fake_cuda.log.count('end') == 2
    assert seg._cur is None and seg.segments == []
    assert red.on_issue is None and red.resets >= 1


def test_capture_segments_in_order(fake_cuda):
    red = _FakeReducer()
    seg = step_graph.SegmentedStepGraph(red, 'cpu')

    def body(before_backward):
        seg._seed = None
        seg._end('forward')
        seg._begin()
        seg.cut(1)
        seg._end('backward')
        return {'l_pix': 0.0}

    out = seg.capture(body, lambda: None)
    assert out == {'l_pix': 0.0}
    assert [k for _, _, k in seg.segments] == ['forward', 'backward', 'backward', 'optimizer']
    assert seg.segments[1][1] == [(1, 'backward')]
    assert fake_cuda.log.count('begin') == fake_cuda.log.count('end') == 4
    # thread-local capture: RCCL's watchdog thread may poll events while a segment is captured
    assert set(fake_cuda.modes) == {'thread_local'}
