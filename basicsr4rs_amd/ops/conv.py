"""3x3 convolution ops on NHWC feature maps, backed by libsr_hip (csrc/conv3x3.hip).

These replace the cuDNN ``nn.Conv2d(C, C', 3, 1, 1)`` calls of the reference SR nets
(basicsr/archs/arch_util.py:78-79, 135-139; edsr_arch.py:44-48; rcan_arch.py:40-42;
rrdbnet_arch.py:21-25).  Parameters stay the reference's ``nn.Conv2d`` parameters
(``weight`` [Cout, Cin, 3, 3] fp32, ``bias`` [Cout]) so state_dict keys and init match;
their GEMM images (forward rows, flipped dgrad rows, bias in GEMM order) are prepared by
a HIP kernel once per parameter update and cached.

Feature maps inside the nets are NHWC tensors ``[N, H, W, Cp]`` with Cp = channels padded
to a multiple of 8 (padded channels are exactly zero).  Compute dtype: bf16 when CUDA
autocast is enabled (the reference's AMP path, basicsr/models/srrs_model.py:28-31, uses
fp16; bf16 is the documented divergence), fp32 otherwise.
"""
import ctypes
import weakref
import math


import torch

from .. import _lib
from ..utils import ktrace
from .._switches import switch

_PARAM_EPOCH = [0]  # bumped by optimizers that update parameters behind autograd's back


def bump_param_epoch():
    _PARAM_EPOCH[0] += 1


# Weight gradients on a side stream.  Inside ``async_wgrad()`` (the model's backward), every
# conv / linear weight gradient that accumulates straight into a FlatParams .grad is launched on a
# per-device side stream forked from the current stream: its split-K kernel and slab reduce then
# overlap the dgrad chain of the main stream (dgrad i and wgrad i only share their inputs), filling
# kernel tails and the memory-bound reduce under MFMA-bound dgrads.  Operands are record_stream'ed
# to the side stream; leaving the context joins it (the current stream waits on it), so the
# optimizer, the bucketed all-reduce and any reader of .grad see finished gradients.  Results are
# the same kernels on the same inputs: bitwise equal to the single-stream order.
# ``hold`` keeps every side-stream dy alive until the join: autograd accumulates a tensor's two
# gradient contributions IN PLACE into one of them when it holds the last reference (e.g. a conv
# output that is also a residual: RCAN / SwinIR body convs, RSTB convs), and that write on the main
# stream could land while the side-stream weight gradient still reads the buffer (record_stream only
# guards reuse after free).  A second reference makes that accumulation out of place.
_ASYNC = {'depth': 0, 'streams': {}, 'used': False, 'mode': True, 'hold': []}


def _side_stream(device):
    st = _ASYNC['streams'].get(device)
    if st is None:
        st = _ASYNC['streams'][device] = torch.cuda.Stream(device)
    return st


def async_side_stream(device=None):
    """The side stream weight gradients are queued on right now (None outside async_wgrad)."""
    if _ASYNC['depth'] == 0:
        return None
    return _side_stream(device if device is not None else torch.device('cuda', torch.cuda.current_device()))


def async_mode():
    """True (whole weight gradients on the side stream), 'reduce' (only their slab reduces), or
    None outside async_wgrad."""
    return _ASYNC['mode'] if _ASYNC['depth'] > 0 else None


class async_wgrad:
    """Context: weight gradients on the side stream, joined into the current stream on exit.
    ``enabled='reduce'`` moves only the split-K slab reduces there (the slab kernel stays on the
    main stream): a memory-bound reduce then fills the CUs beside the next MFMA-bound conv.
    ``blocks``: blocks whose side-stream launches share one fork inside this context (side_batch;
    None keeps the enclosing / SR_SIDE_BATCH setting).  It is restored on exit, so one model's
    setting never leaks into another's backward."""

    def __init__(self, enabled=True, blocks=None):
        self.enabled = enabled
        self.blocks = blocks
        self._prev_mode = None
        self._prev_k = None

    def __enter__(self):
        if self.enabled:
            _ASYNC['depth'] += 1
            self._prev_mode = _ASYNC['mode']
            _ASYNC['mode'] = self.enabled
            if self.blocks is not None:
                self._prev_k = _SIDE['k']
                _SIDE['k'] = max(0, int(self.blocks))
        return self

    def __exit__(self, exc_type, *exc):
        if self.enabled:
            if exc_type is None:
                side_flush_pending()  # launches still queued by side_batch fork before the join
            else:  # backward failed: its queued gradient launches and callbacks are dropped; a DDP
                # reducer is then mid-step -- the models call GradBucketReducer.abandon_step()
                _SIDE['items'], _SIDE['blocks'] = [], 0
            if self._prev_k is not None:
                _SIDE['k'], self._prev_k = self._prev_k, None
            _ASYNC['depth'] -= 1
            _ASYNC['mode'] = self._prev_mode  # a nested context must not leak its mode outward
            for st in _ASYNC['streams'].values():
                torch.cuda.current_stream(st.device).wait_stream(st)
            if _ASYNC['depth'] == 0:
                _ASYNC['hold'].clear()  # joined: the side stream's reads are ordered before any later write
        return False


# Batched forks (side_batch): inside the context, side-stream launches are queued and forked from
# the current stream ONCE at exit (one event wait for all of them instead of one per launch).  A
# captured step turns every fork into a cross-queue graph edge, and RCAN's 2.5 k-node step spent
# ~2.6 us per node between short kernels; SR_SIDE_BATCH=0 forks per launch (A/B).
# k > 1 (async_wgrad(blocks=k), SR_SIDE_BATCH=k) forks once per k blocks (the queue is flushed at
# the latest by the join).
_SIDE_BATCH = []
_SIDE = {'items': [], 'blocks': 0, 'k': max(0, int(switch('SR_SIDE_BATCH') or 1))}


class side_batch:
    """Context: defer the side-stream launches issued inside (side_launch) to one fork at exit."""

    def __enter__(self):
        self._on = bool(_SIDE['k'])
        if self._on:
            _SIDE_BATCH.append([])
        return self

    def __exit__(self, exc_type, *exc):
        if self._on:
            items = _SIDE_BATCH.pop()
            if exc_type is not None:
                return False
            if _SIDE_BATCH:  # nested: hand over to the enclosing batch
                _SIDE_BATCH[-1].extend(items)
                return False
            _SIDE['items'].extend(items)
            _SIDE['blocks'] += 1
            if _SIDE['blocks'] >= _SIDE['k']:
                side_flush_pending()
        return False


def set_side_batch(k):
    """Default blocks per side-stream fork outside any async_wgrad(blocks=...) (0: fork per launch)."""
    side_flush_pending()
    _SIDE['k'] = max(0, int(k))


def side_batch_blocks():
    return _SIDE['k']


def side_flush_pending():
    """Fork the queued side-stream launches now (the join calls this before waiting)."""
    items = _SIDE['items']
    _SIDE['items'], _SIDE['blocks'] = [], 0
    if items:
        _side_flush(items)


def side_launch(side, fn, tensors=(), hold=None, after=()):
    """Run ``fn`` (kernel launches) on ``side`` after the work queued so far on the current stream:
    ``tensors`` are record_stream'ed there, ``hold`` is kept until the join (_ASYNC['hold']) and
    ``after`` (gradient-ready callbacks) fire once every launch of the fork is queued.  Inside
    side_batch the launch joins the batch's single fork."""
    item = (side, fn, tensors, hold, after)
    if _SIDE_BATCH:
        _SIDE_BATCH[-1].append(item)
    else:  # with whatever earlier blocks left queued, in issue order
        items = _SIDE['items'] + [item]
        _SIDE['items'], _SIDE['blocks'] = [], 0
        _side_flush(items)


def _side_flush(items):
    # Every launch of the fork is queued before ANY gradient-ready callback runs: a callback can
    # complete a bucket, and the segmented DDP capture (utils/step_graph.py) then cuts the graph and
    # rejoins the side stream -- launches still to come in this fork would run outside the capture.
    for side in {id(it[0]): it[0] for it in items}.values():
        side.wait_stream(torch.cuda.current_stream(side.device))
    for side, fn, tensors, hold, after in items:
        for t in tensors:
            if t is not None:
                t.record_stream(side)
        if hold is not None:
            _ASYNC['hold'].append(hold)
        with torch.cuda.stream(side):
            fn()
    for it in items:
        for cb in it[4]:
            cb()


def pad8(c):
    return (c + 7) // 8 * 8


_FP16_WARNED = [False]


def feature_dtype():
    """Compute dtype of the HIP kernels for the current context: bf16 under CUDA autocast of any
    dtype.  The reference's AMP is fp16 + GradScaler (basicsr/models/srrs_model.py:28-31, 79-82);
    the kernels have no fp16 path, so an fp16 autocast request runs in bf16 (same 16-bit storage,
    fp32 range: no loss scaling needed) and says so once per process."""
    if torch.is_autocast_enabled('cuda'):
        if not _FP16_WARNED[0] and torch.get_autocast_dtype('cuda') == torch.float16:
            _FP16_WARNED[0] = True
            import warnings
            warnings.warn('basicsr4rs_amd: autocast asked for float16; the HIP kernels compute in bfloat16 '
                          '(the documented AMP divergence, DESIGN.md §0 / SURVEY.md §0.7)', RuntimeWarning,
                          stacklevel=2)
        return torch.bfloat16
    return torch.float32


class ConvSpec:
    """Static configuration of one conv call (epilogue fusion flags)."""
    __slots__ = ('cin', 'cout', 'cin_p', 'cout_p', 'act', 'slope', 'alpha', 'beta', 'out_ps', 'out_nchw',
                 'aff_scale', 'aff_shift', 'in_up')

    def __init__(self, cin, cout, act=_lib.ACT_NONE, slope=0.0, alpha=1.0, beta=1.0, out_ps=0, out_nchw=False,
                 aff_scale=None, aff_shift=None, cin_p=None, cout_p=None, in_up=0):
        self.cin, self.cout = cin, cout
        self.in_up = in_up
        self.cin_p = cin_p or pad8(cin)
        self.cout_p = cout_p or pad8(cout)
        self.act, self.slope, self.alpha, self.beta = act, float(slope), float(alpha), float(beta)
        self.out_ps, self.out_nchw = out_ps, out_nchw
        self.aff_scale, self.aff_shift = aff_scale, aff_shift
        if out_ps:
            assert cout % (out_ps * out_ps) == 0 and (cout // (out_ps * out_ps)) % 8 == 0, \
                'pixel-shuffled conv needs Cout/r^2 to be a multiple of 8'
            self.cout_p = cout


class _Prep:
    """Cached GEMM images of one (weight, layout) pair and the arguments that rebuild them."""
    __slots__ = ('weight', 'bias', 'dtype', 'shape', 'maps', 'val', 'key', 'used', '__weakref__')


# (id(weight), static key) -> _Prep, WEAK: an entry lives as long as its weight (which holds it in
# weight.__dict__['_sr_prep']) or a batched-refresh table / captured graph that uses it, so weights
# of discarded nets (and their GEMM images) are freed
_PREP_ALL = weakref.WeakValueDictionary()
_PREP_TABLE = {}  # dtype -> (entries, device item table, device block starts, total blocks)
# tables launched by refresh_prepared while a HIP graph was being captured: the graph keeps
# launching the batched refresh on their device buffers, so whoever owns the graph takes these
# references (take_captured_tables) and holds them exactly as long as the graph itself
_CAPTURED_TABLES = []


def _retire_table(dtype):
    # a table not referenced by a captured graph is simply released; one that is stays alive
    # through the graph owner's reference
    _PREP_TABLE.pop(dtype, None)


def take_captured_tables():
    """Device tables of the batched weight-image refresh launched during the capture that just
    ended; the caller keeps them alive with its graph (models/sr_model.py)."""
    out = list(_CAPTURED_TABLES)
    _CAPTURED_TABLES.clear()
    return out


def prepared_images(weight, bias, dtype, shape, maps=(None, None), tag=''):
    """GEMM images (wf, wd, bias_g) of a conv / linear weight, cached until it changes.

    ``shape`` = (cout_real, cin_real, cout_p, cin_p, out_ps, ksize); ``maps`` = device
    (row_map, col_map) or Nones.  A stale entry is rebuilt IN PLACE (captured HIP graphs keep
    pointing at the same buffers); after an optimizer step ``refresh_prepared`` rebuilds every
    image used in the previous step in one launch instead of one per parameter."""
    skey = (dtype, shape, weight.data_ptr(), tag)
    ents = weight.__dict__.setdefault('_sr_prep', {})
    dyn = (weight._version, -1 if bias is None else bias._version, _PARAM_EPOCH[0])
    e = ents.get(skey)
    if e is not None and e.key == dyn:
        e.used = _PARAM_EPOCH[0]
        return e.val
    cout_real, cin_real, cout_p, cin_p, out_ps, ksize = shape
    if e is None:
        dev = weight.device
        taps = 9 if ksize == 3 else 1
        e = _Prep()
        e.weight, e.bias, e.dtype, e.shape, e.maps = weight, bias, dtype, shape, maps
        e.val = (torch.empty(cout_p, taps * cin_p, device=dev, dtype=dtype),
                 torch.empty(cin_p, taps * cout_p, device=dev, dtype=dtype),
                 torch.empty(cout_p, device=dev, dtype=torch.float32))
        ents[skey] = e
        _PREP_ALL[(id(weight), skey)] = e
        _retire_table(dtype)
    wf, wd, bg = e.val
    lib = _lib.load()
    _lib.check(
        lib.sr_conv_prep_mapped(_lib.dtype_code(dtype), ksize, _lib.ptr(weight.detach()),
                                _lib.ptr(bias.detach() if bias is not None else None), cout_real, cin_real, cout_p,
                                cin_p, out_ps, _lib.ptr(maps[0]), _lib.ptr(maps[1]), _lib.ptr(wf), _lib.ptr(wd),
                                _lib.ptr(bg), _lib.stream()))
    e.key, e.used = dyn, _PARAM_EPOCH[0]
    return e.val


def prepared(weight, bias, spec, dtype):
    """GEMM images of a 3x3 conv parameter pair (wf, wd, bias in GEMM order)."""
    return prepared_images(weight, bias, dtype, (spec.cout, spec.cin, spec.cout_p, spec.cin_p, spec.out_ps, 3))


def refresh_prepared():
    """Rebuild, in one launch per dtype, the GEMM images of every weight used during the epoch
    that just ended (call right after ``bump_param_epoch`` by an optimizer step), and re-key
    them to the new epoch so the next forward finds them current.  Graph-capturable."""
    ep = _PARAM_EPOCH[0]
    live = [e for e in _PREP_ALL.values() if e.used == ep - 1]
    if not live:
        return
    lib = _lib.load()
    by_dt = {}
    for e in live:
        by_dt.setdefault(e.dtype, []).append(e)
    for dt, ents in by_dt.items():
        tab = _PREP_TABLE.get(dt)
        if tab is None or tab[0] != ents:
            items = (_lib.PrepItem * len(ents))()
            starts = [0]
            for it, e in zip(items, ents):
                cr, ci, cp, cip, ops, ks = e.shape
                wf, wd, bg = e.val
                it.w, it.bias = e.weight.data_ptr(), (e.bias.data_ptr() if e.bias is not None else None)
                it.Cout_real, it.Cin_real, it.Cout, it.Cin, it.out_ps, it.ksize = cr, ci, cp, cip, ops, ks
                it.row_map = e.maps[0].data_ptr() if e.maps[0] is not None else None
                it.col_map = e.maps[1].data_ptr() if e.maps[1] is not None else None
                it.wf, it.wd, it.bias_g = wf.data_ptr(), wd.data_ptr(), bg.data_ptr()
                starts.append(starts[-1] + lib.sr_conv_prep_blocks(ctypes.byref(it)))
            dev = ents[0].weight.device
            raw = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8).to(dev)
            st = torch.tensor(starts, dtype=torch.int32).to(dev)
            tab = (list(ents), raw, st, starts[-1])
            _retire_table(dt)
            _PREP_TABLE[dt] = tab
        _, raw, st, total = tab
        if torch.cuda.is_current_stream_capturing():
            _CAPTURED_TABLES.append(tab)
        _lib.check(lib.sr_conv_prep_batch(_lib.dtype_code(dt), _lib.ptr(raw), _lib.ptr(st), len(ents), total,
                                          _lib.stream()))
    for e in live:
        e.key = (e.weight._version, -1 if e.bias is None else e.bias._version, ep)
        e.used = ep


def _desc(dtype, N, H, W, cin, ldx, cout, cout_real, ldy, **kw):
    d = _lib.ConvDesc()
    d.dtype = _lib.dtype_code(dtype)
    d.N, d.H, d.W = N, H, W
    d.Cin, d.ldx, d.xcoff, d.in_ps = cin, ldx, kw.get('xcoff', 0), kw.get('in_ps', 0)
    d.Cout, d.Cout_real, d.ldw = cout, cout_real, 9 * cin
    d.ldy, d.ycoff, d.out_ps, d.out_nchw = ldy, kw.get('ycoff', 0), kw.get('out_ps', 0), int(kw.get('out_nchw', 0))
    d.act, d.slope, d.alpha = kw.get('act', 0), kw.get('slope', 0.0), kw.get('alpha', 1.0)
    d.ldg, d.gcoff, d.gate_slope = kw.get('ldg', 0), kw.get('gcoff', 0), kw.get('gate_slope', 0.0)
    d.ldr, d.rcoff, d.beta = kw.get('ldr', 0), kw.get('rcoff', 0), kw.get('beta', 1.0)
    d.ldr2, d.r2coff, d.beta2 = kw.get('ldr2', 0), kw.get('r2coff', 0), kw.get('beta2', 1.0)
    d.rcols, d.in_up = kw.get('rcols', 0), kw.get('in_up', 0)
    d.ksize, d.gate_mode = kw.get('ksize', 3), kw.get('gate_mode', 0)
    d.gcol0, d.gcol1 = kw.get('gcol0', 0), kw.get('gcol1', 0)
    d.ldw = (9 if d.ksize == 3 else 1) * cin
    rs = kw.get('row_scale')
    if rs is not None:
        assert rs.dtype == torch.float32 and rs.is_cuda and rs.numel() == N, 'row_scale: fp32 [N] on the device'
        d.row_scale = rs.data_ptr()
    dot = kw.get('dot')
    if dot is not None:
        assert dot.dtype == dtype and dot.is_contiguous() and dot.shape[:3] == (N, H, W), 'dot: like y'
        d.dot, d.ldd, d.dcoff = dot.data_ptr(), dot.shape[-1], 0
    return d


_DOT_OK = {}


def dot_partials_ok(dtype, N, H, W, cin, cout):
    """Whether a conv (cin -> cout, with a residual) can also emit the partial channel sums of
    y * dot in its epilogue (sr_conv3x3_fwd_dot_ok: the band kernel); cached per shape."""
    key = (dtype, N, H, W, cin, cout, _lib.load().sr_conv3x3_get_variant())
    v = _DOT_OK.get(key)
    if v is None:
        d = _desc(dtype, N, H, W, cin, cin, cout, cout, cout)
        v = _DOT_OK[key] = bool(_lib.load().sr_conv3x3_fwd_dot_ok(d))
    return v


def conv_fwd_raw(x, wf, bias_g, y, N, H, W, cin, cout, cout_real, gate=None, res=None, aff_scale=None,
                 aff_shift=None, res2=None, aux=None, colsum=False, **kw):
    """Launch sr_conv3x3_fwd on already-prepared GEMM weights (shapes checked here).

    ``colsum=True`` also returns the [N, P, cout] fp32 partial channel sums of y (as stored;
    summed over P they are the per-image channel sums): ``(y, parts)``; with ``dot=t`` (bf16, y's
    shape) they are the partial sums of y * t instead (band kernel only, dot_partials_ok)."""
    assert x.is_contiguous() and y.is_contiguous()
    _check_channel_vec(aff_scale, cout_real, 'conv aff_scale')
    _check_channel_vec(aff_shift, cout_real, 'conv aff_shift')
    ldx = kw.pop('ldx', x.shape[-1])
    ldy = kw.pop('ldy', y.shape[-1] if not kw.get('out_nchw') else 0)
    if gate is not None:
        kw.setdefault('ldg', gate.shape[-1])
    if res is not None:
        kw.setdefault('ldr', res.shape[-1])
    if res2 is not None:
        kw.setdefault('ldr2', res2.shape[-1])
    d = _desc(x.dtype, N, H, W, cin, ldx, cout, cout_real, ldy, **kw)
    assert wf.shape[0] >= cout and wf.shape[1] == d.ldw, (wf.shape, cout, cin)
    lib = _lib.load()
    M = N * H * W
    taps = 9 if d.ksize == 3 else 1
    parts = None
    if colsum:
        P = lib.sr_conv3x3_fwd_colsum_parts(d)
        if P <= 0:
            raise ValueError(f'conv3x3_fwd: no fused channel sums for this call (N={N} H={H} W={W} cout={cout})')
        parts = torch.empty(N, P, cout, device=y.device, dtype=torch.float32)
    args = (d, _lib.ptr(x), _lib.ptr(wf), _lib.ptr(bias_g), _lib.ptr(gate), _lib.ptr(res), _lib.ptr(res2),
            _lib.ptr(aff_scale), _lib.ptr(aff_shift), _lib.ptr(y), _lib.ptr(aux), _lib.ptr(parts), _lib.stream())
    keep = (x, wf, bias_g, gate, res, res2, aff_scale, aff_shift, y, aux, parts, kw.get('row_scale'), kw.get('dot'))
    if ktrace.active():
        # algorithmic HBM bytes of the call: x once (pre-upsample size with in_up), the weight image,
        # y as stored (fp32 NCHW for the network tail), every epilogue operand (gate / res / res2 read,
        # aux written: Cout channels per pixel each) and the colsum partial rows
        esz = x.element_size()
        up = d.in_up if d.in_up > 1 else 1
        nbytes = esz * (M // (up * up) * cin + taps * cin * cout)
        nbytes += (4 * M * cout_real) if d.out_nchw else esz * M * cout
        nbytes += esz * M * cout * sum(t is not None for t in (gate, res, res2, aux, kw.get('dot')))
        if parts is not None:
            nbytes += 4 * parts.numel()
        with ktrace.span(lib.sr_conv3x3_fwd_kernel_name(d).decode(), 2.0 * M * taps * cin * cout_real, nbytes,
                         relaunch=lambda a=args, k=keep: lib.sr_conv3x3_fwd(*a), launches=lib.sr_conv3x3_fwd_launches(d)):
            _lib.check(lib.sr_conv3x3_fwd(*args))
    else:
        _lib.check(lib.sr_conv3x3_fwd(*args))
    return (y, parts) if colsum else y


def on_grad_ready(p, fn):
    """Register fn(p), called after a HIP kernel accumulated p's gradient in place (the
    direct-gradient path of conv_wgrad_raw and the LN / attention / CA backwards, which bypass
    autograd's AccumulateGrad).  Kept on the parameter object itself."""
    cbs = p.__dict__.get('_sr_grad_ready')
    if cbs is None:
        cbs = p._sr_grad_ready = []
    cbs.append(fn)


def remove_grad_ready(p, fn):
    """Unregister a callback added by on_grad_ready (no-op if absent)."""
    cbs = p.__dict__.get('_sr_grad_ready')
    if cbs and fn in cbs:
        cbs.remove(fn)


def grad_ready(p):
    for fn in p.__dict__.get('_sr_grad_ready', ()):
        fn(p)


def grad_target(p):
    """The FlatParams gradient view of p (the kernels accumulate the gradient straight into it),
    else None.  If something replaced p.grad since FlatParams bound it (``zero_grad`` with
    set_to_none, an autograd-created tensor), the view is re-bound first, carrying over the
    current gradient value (None = zero), so the optimizer's flat buffer stays authoritative."""
    if p is None or not getattr(p, '_sr_flat', False):
        return None
    view = p._sr_grad_view
    g = p.grad
    if g is None or g.data_ptr() != view.data_ptr():
        with torch.no_grad():
            if g is None:
                view.zero_()
            else:
                view.copy_(g)
        p.grad = view
    return view


def conv_wgrad_raw(dy, x, N, H, W, cin, cin_real, cout, cout_real, scale=1.0, out_ps=0, need_bias=True, params=None,
                   **kw):
    """Weight / bias gradient in the nn.Conv2d parameter layout (fp32).

    With ``params=(weight, bias)`` whose ``.grad`` live in a FlatParams buffer, the reduction
    kernel accumulates into those ``.grad`` views directly (no per-parameter AccumulateGrad
    add kernels), fires the gradient-ready callbacks and returns ``(None, None)`` for autograd.
    """
    tw = tb = None
    if params is not None:
        tw = grad_target(params[0])
        tb = grad_target(params[1]) if need_bias else None
        if tw is None or (need_bias and tb is None):
            tw = tb = None
    d = _lib.WgradDesc()
    d.dtype = _lib.dtype_code(x.dtype)
    d.N, d.H, d.W = N, H, W
    d.Cin, d.Cin_real, d.ldx, d.xcoff = cin, cin_real, kw.get('ldx', x.shape[-1]), kw.get('xcoff', 0)
    d.Cout, d.Cout_real, d.ldy, d.ycoff, d.out_ps = cout, cout_real, kw.get('ldy', dy.shape[-1]), kw.get(
        'ycoff', 0), out_ps
    d.scale = scale
    d.in_up = kw.get('in_up', 0)
    d.ksize = kw.get('ksize', 3)
    lib = _lib.load()
    ws_bytes = lib.sr_conv3x3_wgrad_workspace(d)
    # (a traced step stays single-stream: its per-kernel event spans then time each kernel alone)
    side = async_side_stream(x.device) if tw is not None and not ktrace.active() else None
    if side is not None and async_mode() == 'reduce':  # slab here, its reduce on the side stream
        ws = torch.empty(ws_bytes // 4 + 1, device=x.device, dtype=torch.float32)
        d.accumulate = 1 | 2
        _lib.check(lib.sr_conv3x3_wgrad(d, _lib.ptr(dy), _lib.ptr(x), _lib.ptr(ws), ws_bytes, _lib.ptr(tw), _lib.ptr(tb),
                                        _lib.ptr(kw.get('co_map')), _lib.ptr(kw.get('ci_map')), _lib.stream()))
        d.accumulate = 1
        side_launch(side, lambda: _lib.check(lib.sr_conv3x3_wgrad_reduce(d, _lib.ptr(ws), ws_bytes, _lib.ptr(tw),
                                                                          _lib.ptr(tb), _lib.ptr(kw.get('co_map')),
                                                                          _lib.ptr(kw.get('ci_map')), _lib.stream())),
                    (ws, kw.get('co_map'), kw.get('ci_map')),
                    after=(lambda: grad_ready(params[0]),) + ((lambda: grad_ready(params[1])),) * need_bias)
        return None, None
    if side is not None:  # fork: dy / x are ready on the current stream
        # dy held until the join: no in-place gradient accumulation into it before the side read
        side_launch(side, lambda: _wgrad_launch(lib, d, dy, x, ws_bytes, tw, tb, cin_real, cout_real, need_bias, kw),
                    (dy, x, kw.get('co_map'), kw.get('ci_map')), hold=dy,
                    after=(lambda: grad_ready(params[0]),) + ((lambda: grad_ready(params[1])),) * need_bias)
        return None, None
    return _wgrad_launch(lib, d, dy, x, ws_bytes, tw, tb, cin_real, cout_real, need_bias, kw, params)


def _wgrad_launch(lib, d, dy, x, ws_bytes, tw, tb, cin_real, cout_real, need_bias, kw, params=None):
    N, H, W, cin, cout = d.N, d.H, d.W, d.Cin, d.Cout
    ws = torch.empty(ws_bytes // 4 + 1, device=x.device, dtype=torch.float32)
    kk = 3 if d.ksize == 3 else 1
    if tw is not None:
        d.accumulate = 1
        dw, db = tw, tb
    else:
        dw = torch.empty(cout_real, cin_real, kk, kk, device=x.device, dtype=torch.float32)
        db = torch.empty(cout_real, device=x.device, dtype=torch.float32) if need_bias else None
    M = N * H * W
    args = (d, _lib.ptr(dy), _lib.ptr(x), _lib.ptr(ws), ws_bytes, _lib.ptr(dw), _lib.ptr(db), _lib.ptr(kw.get('co_map')),
            _lib.ptr(kw.get('ci_map')), _lib.stream())
    if ktrace.active():  # the relaunch closure must not accumulate into the live gradients
        scratch = (torch.empty_like(dw), torch.empty_like(db) if db is not None else None)
        rargs = args[:5] + (_lib.ptr(scratch[0]), _lib.ptr(scratch[1])) + args[7:]
        keep = (dy, x, ws, scratch, kw.get('co_map'), kw.get('ci_map'))
        # on the stream current at relaunch time (a side-stream launch is re-timed on the timing stream)
        relaunch = lambda a=rargs, k=keep: lib.sr_conv3x3_wgrad(*a[:-1], _lib.stream())  # noqa: E731
    else:
        relaunch = None
    up = d.in_up if d.in_up > 1 else 1
    # dy and x once, dW / db read-modify-written (accumulate) or written, as fp32
    nbytes = x.element_size() * (M * cout + M // (up * up) * cin) + \
        (8 if tw is not None else 4) * (kk * kk * cin_real * cout_real + (cout_real if need_bias else 0))
    with ktrace.span(lib.sr_conv3x3_wgrad_kernel_name(d).decode() + '+reduce', 2.0 * M * kk * kk * cin_real * cout_real,
                     nbytes, relaunch=relaunch):
        _lib.check(lib.sr_conv3x3_wgrad(*args))
    if tw is not None and params is not None:
        grad_ready(params[0])
        if need_bias:
            grad_ready(params[1])
        return None, None
    return dw, db


def nchw_to_nhwc(x, cp, dtype, shift=None, scale=None):
    N, C, H, W = x.shape
    y = torch.empty(N, H, W, cp, device=x.device, dtype=dtype)
    lib = _lib.load()
    _lib.check(
        lib.sr_nchw_to_nhwc(_lib.dtype_code(dtype), _lib.ptr(x.contiguous()), N, C, H, W, cp, _lib.ptr(shift),
                            _lib.ptr(scale), _lib.ptr(y), _lib.stream()))
    return y


def nhwc_to_nchw(x, c, scale=None, shift=None, coff=0):
    N, H, W, ld = x.shape
    y = torch.empty(N, c, H, W, device=x.device, dtype=torch.float32)
    lib = _lib.load()
    _lib.check(
        lib.sr_nhwc_to_nchw(_lib.dtype_code(x.dtype), _lib.ptr(x), N, H, W, ld, coff, c, _lib.ptr(scale),
                            _lib.ptr(shift), _lib.ptr(y), _lib.stream()))
    return y


def _grid(spec, x):
    """Conv (output) grid of an input map: in_up folds a nearest upsample into the gather."""
    N, H, W, _ = x.shape
    u = spec.in_up if spec.in_up and spec.in_up > 1 else 1
    return N, H * u, W * u


def _out_shape(spec, N, H, W):
    if spec.out_nchw:
        return (N, spec.cout, H, W)
    if spec.out_ps:
        r = spec.out_ps
        return (N, H * r, W * r, spec.cout // (r * r))
    return (N, H, W, spec.cout_p)


def _kpad(spec, dtype, H, W):
    """K-padded weight images (cout_k, cin_k) for a bf16 3x3 conv whose channel counts (as stored) are
    not multiples of 64 but whose output is wide (SwinIR-M's 180 -> 180 convs, stored as 184): with the
    GEMM K padded to 192 (zero weight columns; x rows keep their 184-channel stride, so the last chunk's
    8 extra channels are the next pixel's, times zero) the forward runs on the halo-row 256 x 256 kernel
    with a partial output tile instead of the 64-channel halo kernel.  None otherwise."""
    if (switch('SR_CONV_KPAD') == '0' or dtype != torch.bfloat16 or spec.out_nchw or spec.out_ps
            or (spec.in_up or 1) != 1 or not ((W == 64 and H % 4 == 0) or (W == 128 and H % 2 == 0))):
        return None
    if not (128 <= spec.cin_p and 128 < spec.cout_p < 256) or (spec.cin_p % 64 == 0 and spec.cout_p % 64 == 0):
        return None
    return (spec.cout_p + 63) // 64 * 64, (spec.cin_p + 63) // 64 * 64


def _images(weight, bias, spec, dtype, kp):
    if kp is None:
        return prepared(weight, bias, spec, dtype)
    return prepared_images(weight, bias, dtype, (spec.cout, spec.cin, kp[0], kp[1], spec.out_ps, 3))


class _Conv3x3(torch.autograd.Function):
    """y = beta*res + alpha*act(conv3x3(x) + b), fused pixel-shuffle / NCHW-affine store."""

    @staticmethod
    def forward(ctx, x, res, weight, bias, spec):
        dtype = x.dtype
        N, H, W = _grid(spec, x)
        kp = _kpad(spec, dtype, H, W)
        wf, wd, bg = _images(weight, bias, spec, dtype, kp)
        out_dtype = torch.float32 if spec.out_nchw else dtype
        y = torch.empty(_out_shape(spec, N, H, W), device=x.device, dtype=out_dtype)
        conv_fwd_raw(x, wf, bg, y, N, H, W, kp[1] if kp else spec.cin_p, spec.cout_p, spec.cout, res=res,
                     aff_scale=spec.aff_scale, aff_shift=spec.aff_shift, act=spec.act, slope=spec.slope,
                     alpha=spec.alpha, beta=spec.beta, out_ps=spec.out_ps, out_nchw=spec.out_nchw,
                     in_up=spec.in_up)
        ctx.spec = spec
        # the dgrad stays on the unpadded images: the 158-KB kernel would wait for CUs the side-stream
        # weight gradients hold during backward (DESIGN note 38); the forward has the GPU to itself
        ctx.kp = None
        ctx.has_res = res is not None
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, weight, bias, y if spec.act else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        spec = ctx.spec
        x, weight, bias, y = ctx.saved_tensors
        N, H, W = _grid(spec, x)
        dtype = x.dtype
        alpha = spec.alpha
        if spec.out_nchw:
            assert not spec.act
            scale = spec.aff_scale * alpha if spec.aff_scale is not None else None
            if scale is None and alpha != 1.0:
                scale = torch.full((spec.cout, ), alpha, device=dy.device)
            dY = nchw_to_nhwc(dy, spec.cout_p, dtype, scale=scale)
            alpha = 1.0
        else:
            dY = dy.to(dtype).contiguous()
            if spec.act:
                dY = act_backward(dY, y, spec.act, spec.slope, alpha)
                alpha = 1.0
        _, wd, _ = _images(weight, bias, spec, dtype, ctx.kp)
        dx = dres = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(N, H, W, spec.cin_p, device=x.device, dtype=dtype)
            conv_fwd_raw(dY, wd, None, dx, N, H, W, ctx.kp[0] if ctx.kp else spec.cout_p, spec.cin_p, spec.cin_p,
                         alpha=alpha, in_ps=spec.out_ps, ldx=dY.shape[-1])
            if spec.in_up and spec.in_up > 1:
                dx = nearest_up_backward(dx, spec.in_up)
        if ctx.has_res and ctx.needs_input_grad[1]:
            dres = dy if spec.beta == 1.0 else dy * spec.beta
        if ctx.needs_input_grad[2] or (ctx.has_bias and ctx.needs_input_grad[3]):
            dw, db = conv_wgrad_raw(dY, x, N, H, W, spec.cin_p, spec.cin, spec.cout_p, spec.cout, scale=alpha,
                                    out_ps=spec.out_ps, need_bias=ctx.has_bias, in_up=spec.in_up,
                                    params=(weight, bias))
        return dx, dres, dw, db, None


def conv3x3(x, conv, res=None, **kw):
    """Apply an nn.Conv2d(., ., 3, 1, 1) parameter module to an NHWC feature map."""
    spec = ConvSpec(conv.in_channels, conv.out_channels, **kw)
    return _Conv3x3.apply(x, res, conv.weight, conv.bias, spec)


class _ConvChain(torch.autograd.Function):
    """A chain of 3x3 convs, each activation read only by the next conv: the RRDBNet HR tail
    conv_up1 -> lrelu -> conv_up2 -> lrelu -> conv_hr -> lrelu -> conv_last (rrdbnet_arch.py:112-119),
    with the nearest x2 upsamples folded into conv_up1 / conv_up2's input gather (in_up).

    Forward = the convs of _Conv3x3 back to back.  Backward: a conv's dgrad applies the activation
    derivative of the conv before it in its epilogue (gate = that conv's output, which is this conv's
    input), or -- behind an upsample -- the gated 2x2-sum kernel (sr_nearest_up_backward_gate) does, so
    the chain has no act_backward pass over the HR maps (RRDB x4: 3 per step, 1.1 ms of a 64.5 ms step
    in round 4); each wgrad reads the gated gradient its dgrad also reads.  The activation outputs are
    saved as the next conv's inputs anyway (for its wgrad), so the gates cost no extra memory."""

    @staticmethod
    def forward(ctx, x, specs, *params):
        cur = x
        ins = []
        for i, spec in enumerate(specs):
            w, b = params[2 * i], params[2 * i + 1]
            dtype = cur.dtype
            N, H, W = _grid(spec, cur)
            wf, _, bg = prepared(w, b, spec, dtype)
            y = torch.empty(_out_shape(spec, N, H, W), device=cur.device,
                            dtype=torch.float32 if spec.out_nchw else dtype)
            conv_fwd_raw(cur, wf, bg, y, N, H, W, spec.cin_p, spec.cout_p, spec.cout, aff_scale=spec.aff_scale,
                         aff_shift=spec.aff_shift, act=spec.act, slope=spec.slope, alpha=spec.alpha, beta=spec.beta,
                         out_ps=spec.out_ps, out_nchw=spec.out_nchw, in_up=spec.in_up)
            ins.append(cur)
            cur = y
        ctx.specs = specs
        ctx.save_for_backward(*ins, cur if specs[-1].act else None, *params)
        return cur

    @staticmethod
    def backward(ctx, dy):
        specs = ctx.specs
        L = len(specs)
        saved = ctx.saved_tensors
        ins, y_last, params = saved[:L], saved[L], saved[L + 1:]
        grads = [None] * (2 * L)
        d = dy
        for i in reversed(range(L)):
            spec, xi = specs[i], ins[i]
            w, b = params[2 * i], params[2 * i + 1]
            N, H, W = _grid(spec, xi)
            dtype = xi.dtype
            alpha = spec.alpha
            if spec.out_nchw:
                scale = spec.aff_scale * alpha if spec.aff_scale is not None else None
                if scale is None and alpha != 1.0:
                    scale = torch.full((spec.cout, ), alpha, device=d.device)
                dY = nchw_to_nhwc(d, spec.cout_p, dtype, scale=scale)
                alpha = 1.0
            else:
                dY = d.to(dtype).contiguous()
                if i == L - 1 and spec.act:  # the chain's own output activation: not gated by a successor
                    dY = act_backward(dY, y_last, spec.act, spec.slope, alpha)
                    alpha = 1.0
            _, wd, _ = prepared(w, b, spec, dtype)
            if i > 0 or ctx.needs_input_grad[0]:
                # the previous conv's activation output is this conv's input xi: its derivative gates dx
                gated = i > 0 and bool(specs[i - 1].act)
                pslope = specs[i - 1].slope if gated else 0.0
                dx = torch.empty(N, H, W, spec.cin_p, device=xi.device, dtype=dtype)
                up = spec.in_up and spec.in_up > 1
                conv_fwd_raw(dY, wd, None, dx, N, H, W, spec.cout_p, spec.cin_p, spec.cin_p, alpha=alpha,
                             in_ps=spec.out_ps, ldx=dY.shape[-1], gate=xi if gated and not up else None,
                             gate_slope=pslope)
                if up:
                    dx = nearest_up_backward(dx, spec.in_up, gate=xi if gated else None, slope=pslope)
                d = dx
            # needs_input_grad: (x, specs, w0, b0, w1, b1, ...); a frozen conv pays no weight gradient
            has_b = params[2 * i + 1] is not None
            if ctx.needs_input_grad[2 + 2 * i] or (has_b and ctx.needs_input_grad[3 + 2 * i]):
                grads[2 * i], grads[2 * i + 1] = conv_wgrad_raw(dY, xi, N, H, W, spec.cin_p, spec.cin, spec.cout_p,
                                                                spec.cout, scale=alpha, out_ps=spec.out_ps,
                                                                need_bias=has_b, in_up=spec.in_up, params=(w, b))
        return (d if ctx.needs_input_grad[0] else None, None, *grads)


def conv_chain(x, convs, kws):
    """Apply nn.Conv2d(., ., 3, 1, 1) modules ``convs`` in sequence (keyword sets ``kws``: ConvSpec
    arguments), as one autograd node whose backward fuses each activation derivative into the next
    conv's dgrad (_ConvChain).  Only for chains whose intermediate maps feed nothing else."""
    specs = tuple(ConvSpec(c.in_channels, c.out_channels, **kw) for c, kw in zip(convs, kws))
    if any(sp.out_ps for sp in specs):
        raise ValueError('conv_chain: no pixel-shuffle convs')
    params = []
    for c in convs:
        params += [c.weight, c.bias]
    return _ConvChain.apply(x, specs, *params)


class _ResBlock(torch.autograd.Function):
    """ResidualBlockNoBN (basicsr/archs/arch_util.py:64-88): x + rs * conv2(relu(conv1(x))).

    Forward = 2 fused convs; backward = 2 dgrads (ReLU mask and residual fused in the
    epilogues) + 2 wgrads.  Saves x and t = relu(conv1(x)).
    """

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, spec1, spec2, res_scale):
        dtype = x.dtype
        N, H, W, C = x.shape
        wf1, _, bg1 = prepared(w1, b1, spec1, dtype)
        wf2, _, bg2 = prepared(w2, b2, spec2, dtype)
        t = torch.empty(N, H, W, spec1.cout_p, device=x.device, dtype=dtype)
        conv_fwd_raw(x, wf1, bg1, t, N, H, W, spec1.cin_p, spec1.cout_p, spec1.cout, act=_lib.ACT_RELU)
        y = torch.empty(N, H, W, spec2.cout_p, device=x.device, dtype=dtype)
        conv_fwd_raw(t, wf2, bg2, y, N, H, W, spec2.cin_p, spec2.cout_p, spec2.cout, res=x, alpha=res_scale,
                     beta=1.0)
        ctx.specs = (spec1, spec2)
        ctx.res_scale = res_scale
        ctx.save_for_backward(x, t, w1, b1, w2, b2)
        return y

    @staticmethod
    def backward(ctx, dy):
        with side_batch():  # with side-stream weight gradients: both forked once, after the block
            return _ResBlock._backward_body(ctx, dy)

    @staticmethod
    def _backward_body(ctx, dy):
        x, t, w1, b1, w2, b2 = ctx.saved_tensors
        spec1, spec2 = ctx.specs
        rs = ctx.res_scale
        dtype = x.dtype
        N, H, W, C = x.shape
        dy = dy.to(dtype).contiguous()
        _, wd1, _ = prepared(w1, b1, spec1, dtype)
        _, wd2, _ = prepared(w2, b2, spec2, dtype)
        dz1 = torch.empty_like(t)
        conv_fwd_raw(dy, wd2, None, dz1, N, H, W, spec2.cout_p, spec2.cin_p, spec2.cin_p, alpha=rs, gate=t,
                     gate_slope=0.0)
        dw2, db2 = conv_wgrad_raw(dy, t, N, H, W, spec2.cin_p, spec2.cin, spec2.cout_p, spec2.cout, scale=rs,
                                  params=(w2, b2))
        dx = torch.empty_like(x)
        conv_fwd_raw(dz1, wd1, None, dx, N, H, W, spec1.cout_p, spec1.cin_p, spec1.cin_p, res=dy, beta=1.0)
        dw1, db1 = conv_wgrad_raw(dz1, x, N, H, W, spec1.cin_p, spec1.cin, spec1.cout_p, spec1.cout, scale=1.0,
                                  params=(w1, b1))
        return dx, dw1, db1, dw2, db2, None, None, None


def res_block(x, conv1, conv2, res_scale):
    s1 = ConvSpec(conv1.in_channels, conv1.out_channels, act=_lib.ACT_RELU)
    s2 = ConvSpec(conv2.in_channels, conv2.out_channels, alpha=res_scale)
    return _ResBlock.apply(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, s1, s2, float(res_scale))


def act_backward(dy, y, act, slope, alpha):
    """dz = alpha * dy * act'(.) using the sign of the activation output y (relu/lrelu)."""
    lib = _lib.load()
    out = torch.empty_like(dy)
    _lib.check(
        lib.sr_act_backward(_lib.dtype_code(dy.dtype), _lib.ptr(dy), _lib.ptr(y.contiguous()), dy.numel(), act,
                            float(slope), float(alpha), _lib.ptr(out), _lib.stream()))
    return out


class _ToNHWC(torch.autograd.Function):
    """Network head: NCHW fp32 image -> NHWC feature map, y = (x - shift) * scale."""

    @staticmethod
    def forward(ctx, x, cp, dtype, shift, scale):
        ctx.c = x.shape[1]
        ctx.scale = scale
        return nchw_to_nhwc(x, cp, dtype, shift=shift, scale=scale)

    @staticmethod
    def backward(ctx, dy):
        return nhwc_to_nchw(dy.contiguous(), ctx.c, scale=ctx.scale), None, None, None, None


def _check_channel_vec(v, c, what):
    """A per-channel fp32 vector the kernels index 0 .. c - 1 (a short one would be read past its end)."""
    if v is not None and v.numel() < c:
        raise ValueError(f'{what} has {v.numel()} values for {c} channels')


def to_nhwc(x, cp, dtype, shift=None, scale=None):
    if x.shape[1] > cp:
        raise ValueError('channel padding smaller than the input channels')
    _check_channel_vec(shift, x.shape[1], 'to_nhwc shift')
    _check_channel_vec(scale, x.shape[1], 'to_nhwc scale')
    return _ToNHWC.apply(x.contiguous().float(), cp, dtype, shift, scale)


def vec(values, device):
    """Small per-channel fp32 constant on the device (mean / scale vectors)."""
    return torch.as_tensor(values, dtype=torch.float32).reshape(-1).to(device)


def inv_range(img_range, c, device):
    return torch.full((c, ), 1.0 / img_range, dtype=torch.float32, device=device)


def upsample_specs(scale):
    if (scale & (scale - 1)) == 0:
        return [2] * int(math.log(scale, 2))
    if scale == 3:
        return [3]
    raise ValueError(f'scale {scale} is not supported. Supported scales: 2^n and 3.')


def nearest_up_backward(d, s, out=None, accumulate=False, gate=None, slope=0.0):
    """Sum of each s x s block of an NHWC map (backward of nearest upsampling by s); with ``gate`` (the
    upsampled H x W map, a ReLU / LeakyReLU output) times its activation derivative (gate > 0 ? 1 : slope)."""
    N, Hs, Ws, C = d.shape
    H, W = Hs // s, Ws // s
    if out is None:
        out = torch.empty(N, H, W, C, device=d.device, dtype=d.dtype)
    if gate is not None and (tuple(gate.shape[:3]) != (N, H, W) or gate.shape[-1] < C or gate.dtype != d.dtype
                             or not gate.is_contiguous()):
        raise ValueError(f'nearest_up_backward: gate {tuple(gate.shape)} {gate.dtype} for {(N, H, W, C)} {d.dtype}')
    lib = _lib.load()
    _lib.check(lib.sr_nearest_up_backward_gate(_lib.dtype_code(d.dtype), _lib.ptr(d), C, N, H, W, C, s, _lib.ptr(gate),
                                               gate.shape[-1] if gate is not None else 0, float(slope), _lib.ptr(out),
                                               out.shape[-1], int(accumulate), _lib.stream()))
    return out


class _ToNCHW(torch.autograd.Function):
    """NHWC feature map -> NCHW fp32, y = x*scale[c] + shift[c] (first c channels)."""

    @staticmethod
    def forward(ctx, x, c, scale, shift):
        ctx.c, ctx.cp, ctx.scale, ctx.dtype = c, x.shape[-1], scale, x.dtype
        return nhwc_to_nchw(x.contiguous(), c, scale=scale, shift=shift)

    @staticmethod
    def backward(ctx, dy):
        return nchw_to_nhwc(dy.contiguous(), ctx.cp, ctx.dtype, scale=ctx.scale), None, None, None


def to_nchw(x, c, scale=None, shift=None):
    _check_channel_vec(shift, c, 'to_nchw shift')
    _check_channel_vec(scale, c, 'to_nchw scale')
    return _ToNCHW.apply(x, c, scale, shift)
