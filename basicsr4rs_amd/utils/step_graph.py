"""The distributed train step as a chain of HIP graphs, cut at the gradient buckets.

The single-process step is one captured HIP graph (models/sr_model.py).  With DDP the step holds
collectives whose timing matters -- each bucket's all-reduce should start as soon as backward has
produced that bucket (basicsr/models/base_model.py:87-105 via torch DDP) -- and an eager step is
host-bound on launch-heavy nets (RCAN: 2.7 k launches, 54.5 ms eager against 36.5 ms replayed).
So the step is captured as segments sharing one memory pool:

    seg 0: forward, loss, backward up to the point where bucket b0 is complete
    seg 1: backward until bucket b1 is complete
    ...
    seg k: the rest of backward
    opt:   fused Adam + EMA + weight-image refresh

``GradBucketReducer.on_issue`` is pointed at ``cut`` during capture: the reducer reports a ready
bucket from its gradient-ready callback, which ends the current segment (after joining the
side-stream weight-gradient work into the capture stream) and begins the next.  ``replay`` runs
each segment and, right after it, launches the all-reduces of the buckets that segment completed:
RCCL orders them after the segment on its own stream while the next segment's kernels run, so the
exchange overlaps backward exactly as in the eager step, with no per-kernel host work.  After the
last backward segment the remaining buckets go out, the step joins them (stream waits) and replays
the optimizer segment.  Segments replay in capture order, which is what sharing one pool requires.

Every segment starts with one tiny kernel, so that two cuts with nothing launched between them
(a conv's weight and bias straddling a bucket boundary) never produce an empty graph.
"""
import torch

from ..ops.conv import _ASYNC


class SegmentedStepGraph:

    def __init__(self, reducer, device):
        self.red = reducer
        self.pool = torch.cuda.graph_pool_handle()
        self.segments = []  # (graph, buckets completed by it, 'backward' | 'wait')
        self._cur = None
        self._cur_buckets = []
        self._tick = torch.zeros(1, device=device, dtype=torch.int32)
        self.stream = torch.cuda.Stream(device)

    # ---- capture -------------------------------------------------------------------------
    def _begin(self):
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self.pool)
        self._tick.add_(1)  # the segment's first node
        self._cur, self._cur_buckets = g, []

    def _end(self, when):
        cur = torch.cuda.current_stream()
        for st in _ASYNC['streams'].values():  # rejoin side streams forked during this segment
            cur.wait_stream(st)
        self._cur.capture_end()
        self.segments.append((self._cur, self._cur_buckets, when))
        self._cur = None

    def cut(self, b):
        """GradBucketReducer.on_issue during capture: bucket b is complete here."""
        self._cur_buckets.append(b)
        self._end('backward')
        self._begin()

    def capture(self, backward_fn, optimizer_fn):
        """Capture backward_fn() (forward + loss + backward; returns the loss dict) cut at the ready
        buckets, then optimizer_fn() as the last segment.  Returns backward_fn's result."""
        torch.cuda.synchronize()
        self.stream.wait_stream(torch.cuda.current_stream())
        self.red.on_issue = self.cut
        try:
            with torch.cuda.stream(self.stream):
                self._begin()
                out = backward_fn()
                # buckets whose parameters did not all report ready go out after the last
                # backward segment (every rank issues the same collectives)
                self._cur_buckets = []
                flushed = []
                self.red.on_issue = flushed.append
                self.red.flush()
                self._cur_buckets = flushed
                self._end('wait')
                self._begin()
                optimizer_fn()
                self._end('optimizer')
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
        for g, buckets, when in self.segments:
            if when == 'optimizer':
                for h in red.handles:
                    h.wait()
                red.last_issue_log, red.issue_log = red.issue_log, []
                red.reset()
            g.replay()
            for b in buckets:
                red.all_reduce_bucket(b)
                red.issued[b] = True
                red.issue_log.append((b, when))

    @property
    def n_segments(self):
        return len(self.segments)
