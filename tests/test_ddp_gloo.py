"""Multi-process gradient reduction (the DDP path, basicsr/models/base_model.py:87-105) on
CPU with the gloo backend, world_size 2: the bucketed reducer launched from backward hooks
must reproduce the full-batch gradient (mean over ranks = DDP average)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basicsr4rs_amd.utils.flat import FlatParams, GradBucketReducer


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _net():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(), torch.nn.Conv2d(8, 8, 3, padding=1),
                               torch.nn.ReLU(), torch.nn.Conv2d(8, 3, 3, padding=1))


def _worker(rank, world, port, bucket_mb, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    net = _net()
    flat = FlatParams(net)
    red = GradBucketReducer(flat, bucket_mb=bucket_mb)
    red.broadcast_params(0)
    g = torch.Generator().manual_seed(123)
    x = torch.randn(4, 3, 8, 8, generator=g)
    y = torch.randn(4, 3, 8, 8, generator=g)
    for step in range(2):
        flat.zero_grad()
        sl = slice(rank * 2, rank * 2 + 2)
        ((net(x[sl]) - y[sl])**2).mean().backward()
        red.wait()
        grads = (flat.grad / world).clone()
    if rank == 0:
        # buckets tile the flat gradient; the one issued last holds the first parameters
        spans = sorted((lo, hi) for lo, hi, _ in red.buckets)
        assert spans[0][0] == 0 and spans[-1][1] == flat.offsets[-1]
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert 0 in red.buckets[-1][2] and red.buckets[-1][0] == 0
        # every bucket issued from the post-accumulate hooks while backward ran, not at the join
        assert sorted(b for b, _ in red.last_issue_log) == list(range(len(red.buckets)))
        assert all(when == 'backward' for _, when in red.last_issue_log), red.last_issue_log
        q.put((grads, len(red.buckets)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('bucket_mb', [25.0, 0.0005])
def test_bucketed_allreduce_matches_full_batch(bucket_mb):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, bucket_mb, q)) for r in range(2)]
    for p in procs:
        p.start()
    grads, nb = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    net = _net()
    g = torch.Generator().manual_seed(123)
    x = torch.randn(4, 3, 8, 8, generator=g)
    y = torch.randn(4, 3, 8, 8, generator=g)
    ref = []
    for xs, ys in ((x[:2], y[:2]), (x[2:], y[2:])):
        net.zero_grad()
        ((net(xs) - ys)**2).mean().backward()
        ref.append(torch.cat([p.grad.reshape(-1) for p in net.parameters()]))
    ref = (ref[0] + ref[1]) / 2
    assert torch.allclose(grads, ref, rtol=1e-5, atol=1e-6)
    if bucket_mb < 0.01:
        assert nb > 1


class _DirectLinear(torch.autograd.Function):
    """y = x W^T whose weight gradient is accumulated straight into the flat .grad view and
    reported through ops.conv.grad_ready (the path of the HIP wgrad kernels), not autograd."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.p = w
        return x @ w.t()

    @staticmethod
    def backward(ctx, gy):
        from basicsr4rs_amd.ops.conv import grad_ready, grad_target
        (x, ) = ctx.saved_tensors
        gx, gw = gy @ ctx.p.detach(), gy.t() @ x
        tgt = grad_target(ctx.p)
        if tgt is None:  # not in a FlatParams (the single-process reference): plain autograd
            return gx, gw
        tgt.add_(gw)
        grad_ready(ctx.p)
        return gx, None


class _TwiceNet(torch.nn.Module):
    """w1 applied twice per step (two gradient contributions), w2 once."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(1)
        self.w1 = torch.nn.Parameter(torch.randn(16, 16) * 0.3)
        self.w2 = torch.nn.Parameter(torch.randn(4, 16) * 0.3)

    def forward(self, x):
        h = torch.tanh(_DirectLinear.apply(x, self.w1))
        h = torch.tanh(_DirectLinear.apply(h, self.w1))
        return _DirectLinear.apply(h, self.w2)


def _twice_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    net = _TwiceNet()
    flat = FlatParams(net)
    red = GradBucketReducer(flat, bucket_mb=0.0005, last_bucket_mb=0.0005)  # one parameter per bucket
    g = torch.Generator().manual_seed(7)
    x, y = torch.randn(8, 16, generator=g), torch.randn(8, 4, generator=g)
    sl = slice(rank * 4, rank * 4 + 4)
    out = []
    for step in range(3):
        flat.zero_grad()
        ((net(x[sl]) - y[sl])**2).mean().backward()
        red.wait()
        out.append(((flat.grad / world).clone(), list(red.last_issue_log)))
    if rank == 0:
        q.put((out, red.expected))
    dist.barrier()
    red.remove()
    flat.zero_grad()
    ((net(x[sl]) - y[sl])**2).mean().backward()  # no hooks left: nothing issued, nothing raised
    assert red.issue_log == []
    dist.destroy_process_group()


def test_reducer_counts_repeated_contributions():
    """a parameter with two gradient contributions per step must not have its bucket
    all-reduced after the first one.  The first step learns the counts (w1: 2 direct + the autograd hook, w2: 1 + hook) and joins
    every bucket; later steps issue each bucket during backward only after its last contribution;
    the averaged gradient equals the full-batch gradient every step."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_twice_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out, expected = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert expected == [3, 2]  # + autograd's post-accumulate hook (it fires for a None gradient too)
    net = _TwiceNet()
    g = torch.Generator().manual_seed(7)
    x, y = torch.randn(8, 16, generator=g), torch.randn(8, 4, generator=g)
    ref = []
    for sl in (slice(0, 4), slice(4, 8)):
        net.zero_grad()
        ((net(x[sl]) - y[sl])**2).mean().backward()
        ref.append(torch.cat([p.grad.reshape(-1) for p in net.parameters()]))
    ref = (ref[0] + ref[1]) / 2
    for step, (grads, log) in enumerate(out):
        assert torch.allclose(grads, ref, rtol=1e-5, atol=1e-6), step
        assert all(w == ('wait' if step == 0 else 'backward') for _, w in log), (step, log)


def test_reducer_raises_on_extra_contribution():
    """More contributions than learned on the first step: the reducer raises instead of letting a
    gradient land after its bucket was reduced (world 1, gloo)."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(_free_port())
    dist.init_process_group('gloo', rank=0, world_size=1)
    try:
        net = _TwiceNet()
        flat = FlatParams(net)
        red = GradBucketReducer(flat, bucket_mb=0.0005, last_bucket_mb=0.0005)
        x = torch.randn(2, 16)
        flat.zero_grad()
        net(x).sum().backward()
        red.wait()
        assert red.expected == [3, 2]
        flat.zero_grad()
        h = _DirectLinear.apply(torch.tanh(_DirectLinear.apply(x, net.w1)), net.w1)
        h = _DirectLinear.apply(torch.tanh(h), net.w1)  # a third use of w1
        with pytest.raises(RuntimeError, match='more than the 3'):
            _DirectLinear.apply(h, net.w2).sum().backward()
        red.remove()
    finally:
        dist.destroy_process_group()


def test_reducer_relearns_after_unfreeze():
    """a parameter frozen on the first step (EDVR ``tsa_iter``, BasicVSR ``fix_flow``)
    and unfrozen later must not abort the step: a change of the requires_grad set makes the next
    step a learning step (every bucket at the join), after which buckets go out during backward
    again.  ``find_unused_parameters`` keeps every step at the join (world 1, gloo)."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(_free_port())
    dist.init_process_group('gloo', rank=0, world_size=1)
    try:
        net = _TwiceNet()
        flat = FlatParams(net)
        red = GradBucketReducer(flat, bucket_mb=0.0005, last_bucket_mb=0.0005)
        x = torch.randn(2, 16)
        logs = []
        for step in range(4):
            net.w1.requires_grad_(step >= 1)
            flat.zero_grad()
            net(x).sum().backward()
            red.wait()
            logs.append(sorted(w for _, w in red.last_issue_log))
            if step == 0:
                assert red.expected[0] == 0
        assert red.expected == [3, 2]
        assert logs[1] == ['wait', 'wait'] and logs[2] == ['backward', 'backward'], logs
        red.remove()
        red = GradBucketReducer(flat, bucket_mb=0.0005, last_bucket_mb=0.0005, find_unused=True)
        for step in range(2):
            flat.zero_grad()
            net(x).sum().backward()
            red.wait()
            assert all(w == 'wait' for _, w in red.last_issue_log)
        red.remove()
    finally:
        dist.destroy_process_group()


class _FailOnce(torch.autograd.Function):
    """Identity whose backward raises while ``armed`` (a backward that fails mid-way)."""
    armed = [False]

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if _FailOnce.armed[0]:
            raise RuntimeError('injected backward failure')
        return g


def test_reducer_abandon_step_after_failed_backward():
    """A backward that raises after some buckets went out (the last conv's gradient is complete
    before the failure) leaves the reducer mid-step; ``abandon_step`` joins and resets it, and the
    next step reduces every bucket during backward to the right gradient.  Without it the next
    step's counts run past the learned ones and raise.  World 1 over gloo (one process)."""
    port = _free_port()
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        c1, c2 = torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.Conv2d(8, 3, 3, padding=1)
        net = torch.nn.ModuleList([c1, c2])
        flat = FlatParams(net)
        red = GradBucketReducer(flat, bucket_mb=0.0005)
        x = torch.randn(2, 3, 8, 8)

        def loss():
            return c2(_FailOnce.apply(torch.relu(c1(x)))).square().mean()

        def step(fail=False):
            flat.zero_grad()
            _FailOnce.armed[0] = fail
            try:
                loss().backward()
            finally:
                _FailOnce.armed[0] = False

        step()
        red.wait()  # learning step
        ref = flat.grad.clone()
        with pytest.raises(RuntimeError, match='injected'):
            step(fail=True)
        assert any(when == 'backward' for _, when in red.issue_log)  # c2's bucket already went out
        red.abandon_step()
        step()
        red.wait()
        assert all(when == 'backward' for _, when in red.last_issue_log), red.last_issue_log
        assert torch.equal(flat.grad, ref)
        # without abandon_step the step after a failure over-counts c2's contributions
        with pytest.raises(RuntimeError, match='injected'):
            step(fail=True)
        with pytest.raises(RuntimeError, match='more than'):
            step()
    finally:
        dist.destroy_process_group()
