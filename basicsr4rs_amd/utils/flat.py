"""Flat fp32 parameter / gradient storage, fused Adam+EMA, bucketed gradient all-reduce.

The reference's train step (basicsr/models/sr_model.py:91-118) is: zero_grad, forward, loss,
backward (DDP all-reduce of every gradient, basicsr/models/base_model.py:87-105), Adam step
(torch.optim.Adam, base_model.py:107-124), EMA (base_model.py:75-82).  Here the parameters
of the net (and of its EMA copy) are re-pointed into ONE contiguous fp32 buffer each, and
their ``.grad`` into one contiguous gradient buffer, so that

* the gradient all-reduce runs on contiguous bucket slices of that buffer, launched from
  post-accumulate-grad hooks while backward is still running (RCCL over xGMI when the
  process group is NCCL; gloo on CPU for tests);
* Adam + EMA is ONE HIP kernel over the flat vectors (sr_adam_ema), with the DDP 1/world
  average folded in as a gradient scale.
"""
import math

import torch
import torch.distributed as dist

from .. import _lib
from ..ops.conv import async_side_stream, bump_param_epoch, on_grad_ready, refresh_prepared, remove_grad_ready


def _params(module):
    return [p for p in module.parameters() if p.requires_grad]


class FlatParams:
    """Re-point ``module``'s trainable parameters (and grads) into contiguous fp32 buffers."""

    def __init__(self, module, with_grad=True):
        self.params = _params(module)
        self.numels = [p.numel() for p in self.params]
        self.offsets = [0]
        for n in self.numels:
            self.offsets.append(self.offsets[-1] + n)
        dev = self.params[0].device
        self.flat = torch.empty(self.offsets[-1], dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.offsets[-1], dtype=torch.float32, device=dev) if with_grad else None
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numels):
                self.flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + n].view_as(p)
                if with_grad:
                    p.grad = self.grad[o:o + n].view_as(p)
                    p._sr_grad_view = p.grad
                    p._sr_flat = True  # HIP wgrad kernels accumulate straight into this .grad view

    def view(self, buf, i):
        return buf[self.offsets[i]:self.offsets[i] + self.numels[i]].view_as(self.params[i])

    def zero_grad(self):
        self.grad.zero_()
        for i, p in enumerate(self.params):  # autograd may have replaced a view; restore it
            if p.grad is None or p.grad.data_ptr() != self.grad.data_ptr() + 4 * self.offsets[i]:
                p.grad = p._sr_grad_view


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (no amsgrad / weight decay) as one HIP kernel over a FlatParams.

    ``state_dict()`` has torch.optim.Adam's layout (per-param ``step``, ``exp_avg``,
    ``exp_avg_sq``), so training states saved by the reference load here and vice versa.
    ``step(ema=FlatParams, ema_decay=d)`` also applies the EMA update in the same pass.
    """

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if weight_decay != 0 or amsgrad:
            raise NotImplementedError('FusedAdam: weight_decay / amsgrad are not used by the SR configs')
        super().__init__(flat.params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False))
        self.fp = flat
        self.m = torch.zeros_like(flat.flat)
        self.v = torch.zeros_like(flat.flat)
        self.nstep = 0
        self.grad_scale = 1.0
        # {step, lr, grad_scale} on the device: the update kernel reads them there, so the step
        # can be captured in a HIP graph; lr / grad_scale are re-uploaded only when they change
        self.hyper = torch.zeros(3, dtype=torch.float32, device=flat.flat.device)
        self._hyper_host = None
        self._bind_state()

    def _bind_state(self):
        self._step_t = torch.tensor(float(self.nstep))  # one host 'step' tensor shared by all params
        for i, p in enumerate(self.fp.params):
            self.state[p] = {'step': self._step_t, 'exp_avg': self.fp.view(self.m, i),
                             'exp_avg_sq': self.fp.view(self.v, i)}
        self.hyper[0] = float(self.nstep)

    def zero_grad(self, set_to_none=False):
        self.fp.zero_grad()

    def host_step(self):
        """Host-side part of a step (step count, lr / grad_scale upload when changed).  Runs
        on every step, also before each replay of a captured step (models/sr_model.py)."""
        self.nstep += 1
        g = self.param_groups[0]
        hv = (float(g['lr']), float(self.grad_scale))
        if hv != self._hyper_host:
            self.hyper[1:3].copy_(torch.tensor(hv, dtype=torch.float32), non_blocking=False)
            self._hyper_host = hv
        self._step_t.fill_(float(self.nstep))

    def device_step(self, ema=None, ema_decay=0.0):
        """The device part (graph-capturable): step counter increment + fused Adam/EMA."""
        g = self.param_groups[0]
        b1, b2 = g['betas']
        lib = _lib.load()
        _lib.check(
            lib.sr_adam_ema_dev(_lib.ptr(self.fp.flat), _lib.ptr(self.fp.grad), _lib.ptr(self.m), _lib.ptr(self.v),
                                _lib.ptr(ema.flat if ema is not None else None), self.fp.flat.numel(),
                                _lib.ptr(self.hyper), float(b1), float(b2), float(g['eps']), float(ema_decay),
                                _lib.stream()))
        bump_param_epoch()
        refresh_prepared()  # the next forward's GEMM weight images, one launch

    @torch.no_grad()
    def step(self, closure=None, ema=None, ema_decay=0.0):
        loss = closure() if closure is not None else None
        self.host_step()
        self.device_step(ema, ema_decay)
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = [float(s['step']) for s in self.state.values() if 'step' in s]
        with torch.no_grad():
            for i, p in enumerate(self.fp.params):
                st = self.state[p]
                self.fp.view(self.m, i).copy_(st['exp_avg'])
                self.fp.view(self.v, i).copy_(st['exp_avg_sq'])
        self.nstep = int(max(steps)) if steps else 0
        self._bind_state()


def ema_copy(flat_dst, flat_src, decay):
    """EMA of parameters only (base_model.py:75-82): dst = dst*decay + src*(1-decay)."""
    with torch.no_grad():
        flat_dst.flat.mul_(decay).add_(flat_src.flat, alpha=1 - decay)
    bump_param_epoch()


class GradBucketReducer:
    """Bucketed gradient all-reduce overlapped with backward (DDP semantics: average).

    Buckets are contiguous slices of ``flat.grad`` in reverse parameter order (the order
    backward produces them), ``bucket_mb`` MiB each (DDP default 25), except the bucket of
    the first parameters: backward finishes those last, so their all-reduce cannot overlap
    any compute, and it is capped at ``last_bucket_mb`` (1 MiB, DDP's first-bucket size)
    so that only a short collective is exposed before the optimizer.

    A parameter's gradient arrives as one or more *contributions* per step: a HIP kernel that
    accumulates straight into the flat buffer reports each launch (``ops.conv.grad_ready``: conv /
    linear wgrads, LayerNorm, attention-table and channel-attention backwards), and gradients that
    still go through autograd report through the post-accumulate-grad hook.  A parameter used twice
    in a step (a module applied twice, weight tying) gets two.  The first step is a learning step:
    every contribution is counted and all buckets are reduced at the join (``wait``).  From then on
    a bucket is issued (async, RCCL stream ordered after the producing kernels) as soon as every
    parameter in it has received the number of contributions counted in the first step, while
    backward continues.  A parameter receiving MORE contributions than that raises (its bucket
    may already be on the wire; DDP raises for the same condition unless its graph is static);
    fewer leaves its bucket to the join.  ``wait()`` joins before the optimizer.  ``issue_log``
    records, per step, which buckets were issued during backward ('backward') and which only at the
    join ('wait'); ``last_issue_log`` keeps the log of the step joined last.  The 1/world average is
    left to the optimizer (FusedAdam.grad_scale) so no extra pass over the gradients runs.

    ``on_issue``: when set (HIP-graph capture of a distributed step, models/sr_model.py), a ready
    bucket is handed to it instead of being all-reduced; the capture cuts its graph there and the
    replay all-reduces the bucket between graph segments (``all_reduce_bucket``).
    """

    def __init__(self, flat, group=None, bucket_mb=25.0, last_bucket_mb=1.0, find_unused=False):
        self.flat = flat
        self.group = group
        # find_unused_parameters (basicsr/models/base_model.py:96-99): the set of contributions may
        # change from step to step, so no bucket can be known complete during backward -- every
        # bucket goes out at the join (correct, without overlap)
        self.find_unused = bool(find_unused)
        self._grad_sig = None  # requires_grad of every parameter when ``expected`` was learned
        self.world = dist.get_world_size(group)
        n = len(flat.params)
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        cap_last = max(1, min(cap, int(last_bucket_mb * 1024 * 1024 / 4)))
        # the first parameters (reduced last) fill a small bucket; the rest, walked in backward
        # order, fill bucket_mb buckets
        head = []
        for i in range(n):
            if head and flat.offsets[i + 1] - flat.offsets[0] > cap_last:
                break
            head.append(i)
        self.buckets = []  # (lo, hi, param indices), in issue order
        cur = []
        for i in reversed(range(len(head), n)):
            cur.append(i)
            lo, hi = flat.offsets[min(cur)], flat.offsets[max(cur) + 1]
            if hi - lo >= cap:
                self.buckets.append((lo, hi, list(cur)))
                cur = []
        if cur:
            self.buckets.append((flat.offsets[min(cur)], flat.offsets[max(cur) + 1], list(cur)))
        self.buckets.append((flat.offsets[head[0]], flat.offsets[head[-1] + 1], list(reversed(head))))
        self.bucket_of = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.bucket_of[i] = b
        self.expected = None  # contributions per parameter and step (learned on the first step)
        self.on_issue = None
        self.hooks, self._ready_fns = [], []
        for i, p in enumerate(flat.params):
            fn = self._make_hook(i)
            self.hooks.append(p.register_post_accumulate_grad_hook(fn))
            on_grad_ready(p, fn)
            self._ready_fns.append((p, fn))
        self.issue_log, self.last_issue_log = [], []
        self.reset()

    def remove(self):
        """Detach from the parameters (hooks and gradient-ready callbacks); the reducer is dead."""
        for h in self.hooks:
            h.remove()
        for p, fn in self._ready_fns:
            remove_grad_ready(p, fn)
        self.hooks, self._ready_fns = [], []

    def reset(self):
        self.counts = [0] * len(self.flat.params)
        self.issued = [False] * len(self.buckets)
        self._started = False
        if self.find_unused:
            self.expected = None
        if self.expected is None:
            self.pending = [None] * len(self.buckets)  # learning step: everything at the join
        else:
            self.pending = [sum(1 for i in idx if self.expected[i] > 0) for (_, _, idx) in self.buckets]
        self.handles = []

    def abandon_step(self):
        """Recover after a backward that raised: join the bucket reductions this step already
        issued and reset the per-step contribution counts, so the next step starts clean (without
        it the next step's counts run past the learned ones and raise, or a bucket never completes).
        ``ops.conv.async_wgrad`` drops the failed backward's queued side-stream launches and their
        gradient-ready callbacks, so the counts of such a step are short.  The failed step's
        gradients are partial: zero them before the next step.  As with DDP, every rank must abandon
        the same step (a step that fails on one rank only leaves the collectives unmatched).  The
        models call this when their backward raises (SRModel._step_body)."""
        for h in self.handles:
            h.wait()
        self.issue_log = []
        self.reset()

    def all_reduce_bucket(self, b):
        """Launch the async all-reduce of bucket b on the current stream's order (or from the
        side stream while weight gradients run there)."""
        lo, hi, _ = self.buckets[b]
        g = self.flat.grad[lo:hi]
        side = async_side_stream(g.device) if g.is_cuda else None
        if side is not None:
            # weight gradients are being accumulated on the side stream (ops.conv.async_wgrad):
            # issue from it, after the main stream's gradient kernels so far
            side.wait_stream(torch.cuda.current_stream(g.device))
            with torch.cuda.stream(side):
                self.handles.append(dist.all_reduce(g, group=self.group, async_op=True))
        else:
            self.handles.append(dist.all_reduce(g, group=self.group, async_op=True))

    def _issue(self, b, when):
        self.issued[b] = True
        self.issue_log.append((b, when))
        if self.on_issue is not None:
            self.on_issue(b)
        else:
            self.all_reduce_bucket(b)

    def _make_hook(self, i):

        def hook(_p):
            if not self._started:  # first gradient of this step
                self._started = True
                sig = tuple(p.requires_grad for p in self.flat.params)
                if sig != self._grad_sig and self.expected is not None:
                    # a freeze / unfreeze since the counts were learned (EDVR tsa_iter, BasicVSR
                    # fix_flow) changes which parameters receive gradients: learn them again
                    self.expected = None
                    self.pending = [None] * len(self.buckets)
                self._grad_sig = sig
            self.counts[i] += 1
            if self.expected is None:
                return
            e = self.expected[i]
            if self.counts[i] > e:
                raise RuntimeError(
                    f'GradBucketReducer: parameter {i} received {self.counts[i]} gradient contributions this step, '
                    f'more than the {e} of the first step; its bucket may already be reduced. The set of gradient '
                    f'contributions must be the same every step (DDP static-graph semantics).')
            if self.counts[i] == e:
                b = self.bucket_of[i]
                self.pending[b] -= 1
                if self.pending[b] == 0:
                    self._issue(b, 'backward')

        return hook

    def flush(self):
        """Issue every bucket not issued yet (parameters unused this step, or the learning step) so
        every rank issues the same collectives in the same order."""
        if self.expected is None:
            self.expected = list(self.counts)
        for b in range(len(self.buckets)):
            if not self.issued[b]:
                self._issue(b, 'wait')

    def wait(self):
        """Issue what is left (flush) and join the outstanding bucket reductions."""
        self.flush()
        for h in self.handles:
            h.wait()
        self.last_issue_log, self.issue_log = self.issue_log, []
        self.reset()

    def broadcast_params(self, src=0):
        dist.broadcast(self.flat.flat, src=src, group=self.group)
        bump_param_epoch()


def bucket_count(nbytes, bucket_mb=25.0):
    return max(1, math.ceil(nbytes / (bucket_mb * 1024 * 1024)))
