"""The distributed train step as a chain of HIP graphs, cut at the gradient buckets.

The single-process step is one captured HIP graph (models/sr_model.py).  With DDP the step holds
collectives whose timing matters -- each bucket's all-reduce should start as soon as backward has
produced that bucket (basicsr/models/base_model.py:87-105 via torch DDP) -- and an eager step is
host-bound on launch-heavy nets (RCAN: 2.7 k launches, 54.5 ms eager against 36.5 ms replayed).
So the step is captured as segments sharing one memory pool:

    fwd:   zero_grad, forward, loss                      (captured on the calling thread)
    bwd 1: backward until bucket b0 is complete          (captured on autograd's device thread)
    bwd 2: backward until bucket b1 is complete
    ...
    bwd k: the rest of backward
    opt:   fused Adam + EMA + weight-image refresh         (calling thread)

A stream capture must end on the thread that began it (HIP: hipErrorStreamCaptureWrongThread), and
autograd runs the backward of CUDA tensors on its own device thread.  So the forward segment ends
on the calling thread just before ``backward()``; an identity node on the loss (``_BeginBackward``,
the first node autograd runs) begins the first backward segment on the device thread and queues an
engine callback that ends the last one there when backward completes.  In between,
``GradBucketReducer.on_issue`` points at ``cut``: the reducer reports a ready bucket from its
gradient-ready callback (device thread), which ends the current segment -- after joining the
side-stream weight-gradient work into the capture stream -- and begins the next.

``replay`` runs each segment and, right after it, launches the all-reduces of the buckets that
segment completed: RCCL orders them after the segment on its own stream while the next segment's
kernels run, so the exchange overlaps backward as in the eager step, with no per-kernel host work.
Buckets that were not complete during backward go out after the last backward segment; the step
then joins all of them (stream waits) and replays the optimizer segment.  Segments replay in capture
order, which is what sharing one pool requires.  Every segment starts with one tiny kernel, so that
two cuts with nothing launched between them (a conv's weight and bias in two buckets) never make an
empty graph.
"""

import torch

from ..ops.conv import _ASYNC
from .._switches import switch

_TRACE = switch('SR_STEP_TRACE') or None


class _BeginBackward(torch.autograd.Function):
    """Identity on the loss whose backward (the first backward node) opens the first backward
    segment on autograd's device thread."""

    @staticmethod
    def forward(ctx, loss, seg):
        ctx.seg = seg
        return loss.view_as(loss)

    @staticmethod
    def backward(ctx, g):
        # ``g`` is autograd's ones_like seed, filled eagerly by backward() outside any capture: the
        # captured backward starts from the seed made inside the forward segment instead
        seg = ctx.seg
        seg._begin()
        torch.autograd.Variable._execution_engine.queue_callback(lambda: seg._end('backward'))
        return seg._seed, None


class SegmentedStepGraph:

    def __init__(self, reducer, device):
        self.red = reducer
        self.pool = torch.cuda.graph_pool_handle()
        self.segments = []  # [graph, [(bucket, 'backward' | 'wait')] to reduce after it, 'forward' | 'backward' | 'optimizer']
        self._cur = None
        self._cur_buckets = []
        self._tick = torch.zeros(1, device=device, dtype=torch.int32)
        self.stream = torch.cuda.Stream(device)

    # ---- capture -------------------------------------------------------------------------
    def _begin(self):
        assert self._cur is None, 'segment already open'
        with torch.cuda.stream(self.stream):
            g = torch.cuda.CUDAGraph()
            # thread-local capture mode: RCCL's watchdog thread polls its collectives' events
            # (hipEventQuery) while a segment is being captured; in the default global mode that
            # poll fails with 'operation not permitted when stream is capturing' and the
            # watchdog aborts the process (seen with --ddp at world 1, round 4)
            g.capture_begin(pool=self.pool, capture_error_mode='thread_local')
            self._tick.add_(1)  # the segment's first node
        self._cur, self._cur_buckets = g, []

    def _end(self, kind):
        with torch.cuda.stream(self.stream):
            for st in _ASYNC['streams'].values():  # rejoin side streams forked during this segment
                self.stream.wait_stream(st)
            self._cur.capture_end()
        self.segments.append([self._cur, self._cur_buckets, kind])
        self._cur = None

    def _abandon(self):
        """An exception inside ``capture``: end the open segment's capture (its graph and every
        segment so far are dropped), so the capture stream is not left in capture mode and later
        CUDA work does not fail with capture-state errors on top of the original one."""
        g, self._cur = self._cur, None
        if g is not None:
            try:
                with torch.cuda.stream(self.stream):
                    for st in _ASYNC['streams'].values():
                        self.stream.wait_stream(st)
                    g.capture_end()
            except RuntimeError:  # invalidated capture (or begun on autograd's thread): nothing to keep
                pass
        self.segments = []
        self._cur_buckets = []
        self.red.reset()

    def cut(self, b):
        """GradBucketReducer.on_issue during capture: bucket b is complete here."""
        self._cur_buckets.append((b, 'backward'))
        self._end('backward')
        self._begin()

    def _before_backward(self, loss):
        with torch.cuda.stream(self.stream):
            self._seed = torch.ones_like(loss)  # in the forward segment: a pool tensor refilled per replay
        self._end('forward')
        self.red.on_issue = self.cut
        return _BeginBackward.apply(loss, self)

    def capture(self, step_body, optimizer_fn):
        """Capture ``step_body(before_backward)`` (forward + loss + backward; returns the loss dict)
        cut at the ready buckets, then ``optimizer_fn()`` as the last segment."""
        torch.cuda.synchronize()
        self.stream.wait_stream(torch.cuda.current_stream())
        try:
            with torch.cuda.stream(self.stream):
                self._begin()
                out = step_body(self._before_backward)
                assert self._cur is None and self.segments[-1][2] == 'backward', 'backward segment left open'
                # buckets whose parameters did not all report ready go out after the last backward
                # segment (every rank issues the same collectives)
                flushed = []
                self.red.on_issue = flushed.append
                self.red.flush()
                self.segments[-1][1].extend((b, 'wait') for b in flushed)
                self._begin()
                optimizer_fn()
                self._end('optimizer')
        except BaseException:
            self._abandon()
            raise
        finally:
            self.red.on_issue = None
        torch.cuda.current_stream().wait_stream(self.stream)
        # the capture issued nothing: clear the reducer's bookkeeping of that step
        self.red.issue_log = []
        self.red.reset()
        return out

    # ---- replay --------------------------------------------------------------------------
    def replay(self):
        red = self.red
        tr = _TRACE and [('start', self._stamp())]
        for i, (g, buckets, kind) in enumerate(self.segments):
            if kind == 'optimizer':
                for h in red.handles:
                    h.wait()
                if tr is not None:
                    tr.append(('join', self._stamp()))
                red.last_issue_log, red.issue_log = red.issue_log, []
                red.reset()
            g.replay()
            if tr is not None:
                tr.append((f'seg{i}:{kind}', self._stamp()))
            for b, when in buckets:
                red.all_reduce_bucket(b)
                red.issued[b] = True
                red.issue_log.append((b, when))
                if tr is not None:
                    tr.append((f'ar{b}', self._stamp()))
        if tr is not None:
            self.trace.append(tr)

    # SR_STEP_TRACE=host: host time after each segment launch / all-reduce issue / join;
    # SR_STEP_TRACE=sync: the same after a device synchronize (per-phase GPU time, no overlap)
    trace = []

    @staticmethod
    def _stamp():
        import time
        if _TRACE == 'sync':
            torch.cuda.synchronize()
        return time.perf_counter()

    @property
    def n_segments(self):
        return len(self.segments)
