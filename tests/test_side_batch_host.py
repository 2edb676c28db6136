"""Host-side semantics of the batched side-stream forks (ops.conv.side_batch / side_launch,
DESIGN.md note 22) with the stream calls stubbed, so it runs without a GPU: launches queued inside
a batch fork once at its exit, in issue order, each one's gradient-ready callbacks after its
launch; nested batches hand over to the outer one; k blocks per fork; the join flushes what is
still queued; without a batch a launch forks at once (after anything queued earlier)."""
import contextlib

import pytest

from basicsr4rs_amd.ops import conv as C


class _Stream:
    device = 'dev'

    def __init__(self, log):
        self.log = log

    def wait_stream(self, other):
        self.log.append('fork')


class _T:
    def __init__(self, log, name):
        self.log, self.name = log, name

    def record_stream(self, s):
        self.log.append('rec:' + self.name)


@pytest.fixture
def stubs(monkeypatch):
    log = []
    monkeypatch.setattr(C.torch.cuda, 'current_stream', lambda device=None: 'main')
    monkeypatch.setattr(C.torch.cuda, 'stream', lambda s: contextlib.nullcontext())
    monkeypatch.setattr(C, '_ASYNC', {'depth': 0, 'streams': {}, 'used': False, 'mode': True, 'hold': []})
    C.set_side_batch(1)
    yield log, _Stream(log)
    C.set_side_batch(1)


def _launch(side, log, name):
    C.side_launch(side, lambda: log.append('run:' + name), (_T(log, name),), hold=name,
                  after=(lambda: log.append('ready:' + name),))


def test_batch_forks_once_in_issue_order(stubs):
    log, side = stubs
    with C.side_batch():
        _launch(side, log, 'a')
        _launch(side, log, 'b')
        assert log == []  # nothing forked yet
    # every launch of the fork is queued before any gradient-ready callback runs (a callback may
    # cut the segmented DDP capture and rejoin the side stream)
    assert log == ['fork', 'rec:a', 'run:a', 'rec:b', 'run:b', 'ready:a', 'ready:b']
    assert C._ASYNC['hold'] == ['a', 'b']


def test_nested_batches_fork_at_the_outer_exit(stubs):
    log, side = stubs
    with C.side_batch():
        _launch(side, log, 'a')
        with C.side_batch():
            _launch(side, log, 'b')
        assert log == []
    assert log.count('fork') == 1 and [x for x in log if x.startswith('run')] == ['run:a', 'run:b']


def test_k_blocks_per_fork_and_join_flush(stubs):
    log, side = stubs
    C.set_side_batch(3)
    for name in 'abcd':
        with C.side_batch():
            _launch(side, log, name)
    # a, b, c forked together after the third block; d still queued
    assert log.count('fork') == 1 and 'run:d' not in log
    with C.async_wgrad(True):
        pass  # the join forks what is still queued before waiting on the side streams
    assert log.count('fork') == 2 and log[-1] == 'ready:d'


def test_unbatched_launch_forks_after_queued_ones(stubs):
    log, side = stubs
    C.set_side_batch(2)
    with C.side_batch():
        _launch(side, log, 'a')
    _launch(side, log, 'b')  # outside any batch: forks now, 'a' first
    assert [x for x in log if x.startswith('run')] == ['run:a', 'run:b'] and log.count('fork') == 1


def test_context_blocks_are_scoped(stubs):
    log, side = stubs
    assert C.side_batch_blocks() == 1
    with C.async_wgrad(True, blocks=3):
        assert C.side_batch_blocks() == 3
        for name in 'ab':
            with C.side_batch():
                _launch(side, log, name)
        assert log == []  # 2 of 3 blocks queued
    assert C.side_batch_blocks() == 1  # restored: no leak into other models
    assert log.count('fork') == 1 and log[-1] == 'ready:b'


def test_exception_in_backward_drops_queued_launches(stubs):
    log, side = stubs
    with pytest.raises(RuntimeError):
        with C.async_wgrad(True, blocks=4):
            with C.side_batch():
                _launch(side, log, 'a')
            raise RuntimeError('backward failed')
    assert log == [] and C._SIDE['items'] == [] and C.side_batch_blocks() == 1


def test_callback_cut_does_not_split_a_fork(stubs):
    log, side = stubs
    cut = []

    def launch(name):
        C.side_launch(side, lambda: log.append('run:' + name), (), after=(lambda: cut.append(list(log)),))

    with C.side_batch():
        launch('a')
        launch('b')
    # the first callback (which could end a capture) already sees both launches queued
    assert cut[0] == ['fork', 'run:a', 'run:b']


def test_exception_inside_batch_drops_its_launches(stubs):
    log, side = stubs
    with pytest.raises(RuntimeError):
        with C.side_batch():
            _launch(side, log, 'a')
            raise RuntimeError('backward failed')
    assert log == []
