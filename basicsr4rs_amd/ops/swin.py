"""SwinIR token ops on the HIP engine (csrc/swin.hip + 1x1 implicit-GEMM linears).

The token map of SwinIR ([B, H*W, C] after PatchEmbed, basicsr/archs/swinir_arch.py:600-604)
is exactly our NHWC feature map, so PatchEmbed / PatchUnEmbed are free.  A SwinTransformerBlock
(swinir_arch.py:283-323) is ONE autograd Function:

    ln1 = LN(x); qkv = Linear(ln1)            -> [M, 3*nH*hdp]   (heads padded to hdp = 32)
    a   = WindowAttention(qkv)                 (shift / partition / mask / bias in-kernel)
    x2  = x + Linear_proj(a)                   (residual fused in the GEMM epilogue)
    ln2 = LN(x2); h = GELU(Linear_fc1(ln2))    (GELU + pre-activation side output fused)
    out = x2 + Linear_fc2(h)

with a hand-written backward (GELU' fused into fc2's dgrad epilogue, LN residual fused).  In bf16
with window 8 and heads of <= 32 (SwinIR-M / -S / the RS configs) the first three lines run as ONE
kernel (round 4, csrc/swin_fused.hip, ``swin_attn_fused``): LayerNorm, qkv, window attention and proj
+ residual on a two-window token tile in LDS, which also writes what the backward reads (ln1, its
statistics, qkv, the attention output, lse) -- or, without autograd (validation / inference), x2 only.
Linears are 1x1 convs: nn.Linear.weight [out][in] is the 1x1 conv weight; the padded head
layout is produced by index maps in the HIP weight-prep kernel.

Stochastic depth (DropPath, swinir_arch.py:14-40 applied at :320-321): in training the two
residual branches are scaled per sample, x2 = x + s1[n]*proj(a), out = x2 + s2[n]*fc2(h), with
s = floor(keep + U[0,1)) / keep drawn per forward (archs/swinir_arch.py).  The factor rides in
the proj / fc2 GEMM epilogues (sr_conv3x3_desc.row_scale); the backward scales the branch
gradients once (sr_row_scale) and feeds them to both the dgrad and the wgrad.
"""
import torch

from .. import _lib
from ..utils import ktrace
from . import conv as C
from .._switches import switch

GELU = 3
# SR_PARAM_REDUCE_MAIN=1 keeps the LayerNorm / attention-table gradient reduces on the main stream
# under async_wgrad (A/B)
_PARAM_REDUCE_SIDE = switch('SR_PARAM_REDUCE_MAIN') != '1'
# SR_ROWSCALE_UNFUSED=1: the proj-branch stochastic-depth gradient by a separate row-scale pass (A/B)
_ROWSCALE_FUSED = switch('SR_ROWSCALE_UNFUSED') != '1'
# SR_SWIN_FUSED=0: the attention half of a block as three launches (LN+qkv, attention, proj) (A/B)
_SWIN_FUSED = switch('SR_SWIN_FUSED') != '0'


class LinearSpec:
    """GEMM geometry of an nn.Linear on padded token rows, with index maps."""

    def __init__(self, cin, cout, cin_p, cout_p, row_map=None, col_map=None):
        self.cin, self.cout, self.cin_p, self.cout_p = cin, cout, cin_p, cout_p
        self.row_map, self.col_map = row_map, col_map  # GEMM index -> param index (or -1)
        co_map = ci_map = None
        if row_map is not None:
            co_map = [0] * cout
            for n, r in enumerate(row_map):
                if r >= 0:
                    co_map[r] = n
        if col_map is not None:
            ci_map = [0] * cin
            for k, c in enumerate(col_map):
                if c >= 0:
                    ci_map[c] = k
        # identity maps are dropped: the slab reduce then reads 16-B rows instead of gathering
        if co_map is not None and co_map == list(range(cout)):
            co_map = None
        if ci_map is not None and ci_map == list(range(cin)):
            ci_map = None
        self.co_map, self.ci_map = co_map, ci_map
        self._dev = {}

    def maps(self, device):
        key = str(device)
        if key not in self._dev:
            t = lambda v: torch.tensor(v, dtype=torch.int32, device=device) if v is not None else None  # noqa: E731
            self._dev[key] = (t(self.row_map), t(self.col_map), t(self.co_map), t(self.ci_map))
        return self._dev[key]


def qkv_spec(C_, nH, hdp):
    hd = C_ // nH
    rows = [(w * C_ + h * hd + d) if d < hd else -1 for w in range(3) for h in range(nH) for d in range(hdp)]
    return LinearSpec(C_, 3 * C_, C.pad8(C_), 3 * nH * hdp, row_map=rows,
                      col_map=[k if k < C_ else -1 for k in range(C.pad8(C_))])


def proj_spec(C_, nH, hdp):
    hd = C_ // nH
    cols = [(h * hd + d) if d < hd else -1 for h in range(nH) for d in range(hdp)]
    return LinearSpec(C_, C_, nH * hdp, C.pad8(C_), row_map=[n if n < C_ else -1 for n in range(C.pad8(C_))],
                      col_map=cols)


def plain_spec(cin, cout):
    return LinearSpec(cin, cout, C.pad8(cin), C.pad8(cout), row_map=[n if n < cout else -1 for n in range(C.pad8(cout))],
                      col_map=[k if k < cin else -1 for k in range(C.pad8(cin))])


def prepared_linear(weight, bias, spec, dtype):
    """GEMM images of an nn.Linear through the padded-head index maps (1x1 conv layout)."""
    rm, cm, _, _ = spec.maps(weight.device)
    return C.prepared_images(weight, bias, dtype, (spec.cout, spec.cin, spec.cout_p, spec.cin_p, 0, 1), (rm, cm),
                             tag='lin')


def linear_fwd(x, wf, bg, spec, N, H, W, **kw):
    y = torch.empty(N, H, W, spec.cout_p, device=x.device, dtype=x.dtype)
    C.conv_fwd_raw(x, wf, bg, y, N, H, W, spec.cin_p, spec.cout_p, spec.cout_p, ksize=1, **kw)
    return y


def linear_dgrad(dy, wd, spec, N, H, W, **kw):
    dx = torch.empty(N, H, W, spec.cin_p, device=dy.device, dtype=dy.dtype)
    C.conv_fwd_raw(dy, wd, None, dx, N, H, W, spec.cout_p, spec.cin_p, spec.cin_p, ksize=1, **kw)
    return dx


def row_scale(x, scale, HW):
    """out[m] = x[m] * scale[m // HW] over the rows of a dense NHWC map (HIP kernel)."""
    out = torch.empty_like(x)
    M = x.numel() // x.shape[-1]
    lib = _lib.load()
    with ktrace.span('row_scale_kernel', 0.0, 2.0 * x.numel() * x.element_size()):
        _lib.check(lib.sr_row_scale(_lib.dtype_code(x.dtype), _lib.ptr(x), M, x.shape[-1], HW, _lib.ptr(scale),
                                    _lib.ptr(out), _lib.stream()))
    return out


row_scale_ = row_scale  # for layernorm_bwd, whose row_scale parameter shadows the function


def linear_wgrad(dy, x, spec, N, H, W, need_bias=True, params=None):
    _, _, co, ci = spec.maps(dy.device)
    dw, db = C.conv_wgrad_raw(dy, x, N, H, W, spec.cin_p, spec.cin, spec.cout_p, spec.cout, ksize=1, co_map=co,
                              ci_map=ci, need_bias=need_bias, params=params)
    return (dw.reshape(spec.cout, spec.cin) if dw is not None else None), db


def layernorm(x, weight, bias, Creal, eps=1e-5):
    N, H, W, Cp = x.shape
    M = N * H * W
    y = torch.empty_like(x)
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    lib = _lib.load()
    with ktrace.span('ln_fwd_kernel', 0.0, 2.0 * M * Creal * x.element_size()):
        _lib.check(
            lib.sr_layernorm_fwd(_lib.dtype_code(x.dtype), _lib.ptr(x), Cp, _lib.ptr(weight.detach()),
                                 _lib.ptr(bias.detach()), M, Creal, Cp, float(eps), _lib.ptr(y), Cp, _lib.ptr(mean),
                                 _lib.ptr(rstd), _lib.stream()))
    return y, mean, rstd


def linear_ln_fwd(x, weight, bias, Creal, wf, bg, spec, N, H, W, act=0, aux=None, eps=1e-5):
    """Linear(LayerNorm(x)) in one launch (sr_linear_ln_fwd: the LayerNorm runs in the lin
    kernel's prologue on the staged token rows), or None when the call is not on that path
    (fp32 parity mode, shapes past the lin kernel) -- the caller then runs the two ops.
    Returns (y, ln, mean, rstd): ln / mean / rstd are what ``layernorm`` returns."""
    Cp = x.shape[-1]
    if x.dtype != torch.bfloat16 or Cp != spec.cin_p or spec.cin_p > 192 or spec.cout_p > 640:
        return None
    unf = switch('SR_LN_UNFUSED')  # A/B: the standalone LayerNorm kernel + linear ('1': both
    if unf == '1' or (unf == 'fc1' and aux is not None) or (unf == 'qkv' and aux is None):  # or one of them)
        return None
    M = N * H * W
    ln = torch.empty_like(x)
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    y = torch.empty(N, H, W, spec.cout_p, device=x.device, dtype=x.dtype)
    d = C._desc(x.dtype, N, H, W, spec.cin_p, Cp, spec.cout_p, spec.cout_p, spec.cout_p, ksize=1, act=act)
    lib = _lib.load()
    with ktrace.span('conv3x3_lin_kernel+ln', 2.0 * M * spec.cin_p * spec.cout_p,
                     x.element_size() * M * (2 * Cp + spec.cout_p * (2 if aux is not None else 1))):
        _lib.check(
            lib.sr_linear_ln_fwd(d, _lib.ptr(x), _lib.ptr(weight.detach()), _lib.ptr(bias.detach()), Creal, float(eps),
                                 _lib.ptr(ln), _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(wf), _lib.ptr(bg), _lib.ptr(y),
                                 _lib.ptr(aux), _lib.stream()))
    return y, ln, mean, rstd


def _direct(params):
    """The optimizer's flat .grad views of ``params`` when every one has one (kernels then
    accumulate into them and the gradient-ready callbacks fire), else None."""
    if params is None:
        return None
    tg = [C.grad_target(p) for p in params]
    return tg if all(g is not None for g in tg) else None


def layernorm_bwd(dy, x, mean, rstd, weight, Creal, res=None, params=None, row_scale=None):
    """dx, dgamma, dbeta; with ``params=(weight, bias)`` held in a FlatParams buffer the
    parameter gradients are accumulated in place and (dx, None, None) is returned.  With
    ``row_scale`` (fp32 [N]) dx is returned as the pair (dx, dx * row_scale[image]) when the
    kernel writes both in one pass (sr_layernorm_bwd_scaled), else the caller scales."""
    N, H, W, Cp = x.shape
    M = N * H * W
    dx = torch.empty_like(x)
    direct = _direct(params)
    if direct is not None:
        dg, db = direct
    else:
        dg = torch.empty(Creal, device=x.device, dtype=torch.float32)
        db = torch.empty(Creal, device=x.device, dtype=torch.float32)
    lib = _lib.load()
    wsb = lib.sr_layernorm_bwd_workspace(M, Creal)
    ws = torch.empty(wsb // 4 + 1, device=x.device, dtype=torch.float32)
    ldr = res.shape[-1] if res is not None else 0
    # side-stream weight gradients (ops.conv.async_wgrad): the dgamma / dbeta reduce goes there too
    side = C.async_side_stream(x.device) if direct is not None and not ktrace.active() and _PARAM_REDUCE_SIDE else None
    nparts = lib.sr_layernorm_bwd_parts(_lib.dtype_code(x.dtype), M, Cp, Cp, Cp, dy.shape[-1], ldr) if side else 0
    if nparts <= 0:
        side = None
    acc = int(direct is not None) | (2 if side is not None else 0)
    scaled = None
    if row_scale is not None and _ROWSCALE_FUSED and x.dtype == torch.bfloat16 and lib.sr_layernorm_bwd_parts(
            _lib.dtype_code(x.dtype), M, Cp, Cp, Cp, dy.shape[-1], ldr) > 0:
        scaled = torch.empty_like(x)
    with ktrace.span('ln_bwd_kernel', 0.0, (4.0 if res is not None else 3.0) * M * Creal * x.element_size()):
        if scaled is not None:  # the stochastic-depth branch gradient in the same pass
            _lib.check(
                lib.sr_layernorm_bwd_scaled(_lib.dtype_code(x.dtype), _lib.ptr(dy), dy.shape[-1], _lib.ptr(x), Cp,
                                            _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(weight.detach()), M, Creal, Cp,
                                            _lib.ptr(res), ldr, _lib.ptr(dx), Cp, _lib.ptr(dg), _lib.ptr(db), _lib.ptr(ws),
                                            wsb, acc, _lib.ptr(row_scale), H * W, _lib.ptr(scaled), _lib.stream()))
        else:
            _lib.check(
                lib.sr_layernorm_bwd(_lib.dtype_code(x.dtype), _lib.ptr(dy), dy.shape[-1], _lib.ptr(x), Cp, _lib.ptr(mean),
                                     _lib.ptr(rstd), _lib.ptr(weight.detach()), M, Creal, Cp, _lib.ptr(res), ldr,
                                     _lib.ptr(dx), Cp, _lib.ptr(dg), _lib.ptr(db), _lib.ptr(ws), wsb, acc,
                                     _lib.stream()))
    if row_scale is not None:
        dx = (dx, scaled if scaled is not None else row_scale_(dx, row_scale, H * W))
    if side is not None:  # (direct is not None): the gradient-ready callbacks follow the reduce
        C.side_launch(side, lambda: _lib.check(lib.sr_layernorm_bwd_reduce(_lib.ptr(ws), nparts, Creal, _lib.ptr(dg),
                                                                           _lib.ptr(db), 1, _lib.stream())), (ws,),
                      after=tuple((lambda p=p: C.grad_ready(p)) for p in params))
        return dx, None, None
    if direct is not None:
        for p in params:
            C.grad_ready(p)
        return dx, None, None
    return dx, dg, db


class _LayerNorm(torch.autograd.Function):
    """Standalone token LayerNorm (PatchEmbed norm / final norm)."""

    @staticmethod
    def forward(ctx, x, weight, bias, Creal):
        y, mean, rstd = layernorm(x, weight, bias, Creal)
        ctx.Creal = Creal
        ctx.save_for_backward(x, mean, rstd, weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, weight, bias = ctx.saved_tensors
        dx, dg, db = layernorm_bwd(dy.to(x.dtype).contiguous(), x, mean, rstd, weight, ctx.Creal,
                                   params=(weight, bias))
        return dx, dg, db, None


def token_layernorm(x, norm):
    return _LayerNorm.apply(x, norm.weight, norm.bias, norm.normalized_shape[0])


class AttnGeom:

    def __init__(self, dim, nH, ws, shift, hdp=32):
        self.dim, self.nH, self.ws, self.shift, self.hdp = dim, nH, ws, shift, hdp
        self.hd = dim // nH
        self.qkv = qkv_spec(dim, nH, hdp)
        self.proj = proj_spec(dim, nH, hdp)


def attn_flops(g, N, H, W):
    """Algorithmic FLOPs of one window-attention forward: QK^T and AV per (window, head),
    2 * 2 * n^2 * head_dim with n = ws^2 tokens (head_dim unpadded)."""
    n = g.ws * g.ws
    units = N * (H // g.ws) * (W // g.ws) * g.nH
    return 4.0 * units * n * n * g.hd


def window_attn(qkv, g, N, H, W, scale, table):
    out = torch.empty(N, H, W, g.nH * g.hdp, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(N * (H // g.ws) * (W // g.ws) * g.nH * g.ws * g.ws, device=qkv.device, dtype=torch.float32)
    lib = _lib.load()
    with ktrace.span('wattn_fwd_kernel', attn_flops(g, N, H, W), 4.0 * N * H * W * g.dim * qkv.element_size()):
        _lib.check(
            lib.sr_window_attn_fwd(_lib.dtype_code(qkv.dtype), _lib.ptr(qkv), qkv.shape[-1], N, H, W, g.ws, g.shift, g.nH,
                                   g.hd, g.hdp, float(scale), _lib.ptr(table), _lib.ptr(out), out.shape[-1], _lib.ptr(lse),
                                   _lib.stream()))
    return out, lse


def window_attn_bwd(qkv, out, dout, lse, g, N, H, W, scale, table, table_param=None):
    dqkv = torch.empty_like(qkv)
    direct = _direct((table_param,) if table_param is not None else None)
    dtable = direct[0] if direct is not None else torch.empty_like(table)
    lib = _lib.load()
    wsb = lib.sr_window_attn_bwd_workspace(N, H, W, g.ws, g.nH)
    ws = torch.empty(wsb // 4 + 1, device=qkv.device, dtype=torch.float32)
    # side-stream weight gradients (ops.conv.async_wgrad): the table-gradient reduce goes there too
    side = C.async_side_stream(qkv.device) if direct is not None and not ktrace.active() and _PARAM_REDUCE_SIDE else None
    with ktrace.span('wattn_bwd_kernel', 2.5 * attn_flops(g, N, H, W), 9.0 * N * H * W * g.dim * qkv.element_size()):
        _lib.check(
            lib.sr_window_attn_bwd(_lib.dtype_code(qkv.dtype), _lib.ptr(qkv), qkv.shape[-1], _lib.ptr(out), _lib.ptr(dout),
                                   out.shape[-1], _lib.ptr(lse), N, H, W, g.ws, g.shift, g.nH, g.hd, g.hdp, float(scale),
                                   _lib.ptr(table), _lib.ptr(dqkv), _lib.ptr(dtable), _lib.ptr(ws), wsb,
                                   int(direct is not None) | (2 if side is not None else 0), _lib.stream()))
    if side is not None:
        parts = lib.sr_window_attn_bwd_parts(_lib.dtype_code(qkv.dtype), N, H, W, g.ws, g.nH, g.hd, g.hdp, qkv.shape[-1],
                                             out.shape[-1])
        C.side_launch(side, lambda: _lib.check(lib.sr_window_attn_dbias_reduce(_lib.ptr(ws), parts, g.nH, g.ws,
                                                                               _lib.ptr(dtable), 1, _lib.stream())),
                      (ws,), after=(lambda: C.grad_ready(table_param),))
        return dqkv, None
    if direct is not None:
        C.grad_ready(table_param)
        return dqkv, None
    return dqkv, dtable


def attn_block_flops(g, N, H, W):
    """Algorithmic FLOPs of the attention half of a block: qkv and proj linears (unpadded C) and
    QK^T + AV (attn_flops)."""
    M = N * H * W
    return 2.0 * M * g.dim * 3 * g.dim + attn_flops(g, N, H, W) + 2.0 * M * g.dim * g.dim


def swin_attn_fused(x, n1w, n1b, Creal, qwf, qbg, tab, pwf, pbg, s1, g, scale, train):
    """x2 = x + s1 * proj(WindowAttention(qkv(LN1(x)))) in one launch (sr_swin_attn_fused_fwd), or
    None when the call is not on that path (fp32 parity mode, other window / head geometries,
    SR_SWIN_FUSED=0).  Training also returns ln1, mean, rstd, qkv, the attention output and lse
    exactly as the unfused path writes them (the backward is shared)."""
    N, H, W, Cp = x.shape
    lib = _lib.load()
    if not _SWIN_FUSED or not lib.sr_swin_attn_fused_ok(_lib.dtype_code(x.dtype), N, H, W, g.ws, g.nH, g.hd, g.hdp,
                                                       Creal, Cp):
        return None
    M = N * H * W
    dev = x.device
    x2 = torch.empty_like(x)
    ln1 = m1 = r1 = qkv = a = lse = None
    if train:
        ln1 = torch.empty_like(x)
        m1 = torch.empty(M, device=dev, dtype=torch.float32)
        r1 = torch.empty(M, device=dev, dtype=torch.float32)
        qkv = torch.empty(N, H, W, 3 * g.nH * g.hdp, device=dev, dtype=x.dtype)
        a = torch.empty(N, H, W, g.nH * g.hdp, device=dev, dtype=x.dtype)
        lse = torch.empty(N * (H // g.ws) * (W // g.ws) * g.nH * g.ws * g.ws, device=dev, dtype=torch.float32)
    # HBM bytes: x read twice (LayerNorm, residual), x2 written; training also ln1, qkv, attention out
    nbytes = x.element_size() * M * (3 * Cp + ((Cp + 3 * g.nH * g.hdp + g.nH * g.hdp) if train else 0))
    with ktrace.span('swin_attn_block_fwd_kernel', attn_block_flops(g, N, H, W), nbytes):
        _lib.check(
            lib.sr_swin_attn_fused_fwd(_lib.ptr(x), _lib.ptr(n1w.detach()), _lib.ptr(n1b.detach()), Creal, 1e-5,
                                       _lib.ptr(qwf), _lib.ptr(qbg), _lib.ptr(tab), _lib.ptr(pwf), _lib.ptr(pbg),
                                       _lib.ptr(s1), N, H, W, g.shift, g.nH, Cp, float(scale), _lib.ptr(x2),
                                       _lib.ptr(ln1), _lib.ptr(m1), _lib.ptr(r1), _lib.ptr(qkv), _lib.ptr(a),
                                       _lib.ptr(lse), _lib.stream()))
    return x2, ln1, m1, r1, qkv, a, lse


def swin_mlp_fused(x, n2w, n2b, Creal, f1wf, f1bg, fc1s, f2wf, f2bg, s2, train):
    """out = x + s2 * fc2(GELU(fc1(LN2(x)))) in one launch (sr_swin_mlp_fused_fwd), or None off that
    path (fp32, wider maps, SR_SWIN_FUSED=0).  Training also returns ln2, mean, rstd, z and h as the
    lin kernel writes them (the backward is shared)."""
    N, H, W, Cp = x.shape
    lib = _lib.load()
    Hp = fc1s.cout_p
    if not _SWIN_FUSED or Cp != fc1s.cin_p or f2wf.shape[0] != Cp or f2wf.numel() != Cp * Hp or \
            not lib.sr_swin_mlp_fused_ok(_lib.dtype_code(x.dtype), Creal, Cp, Hp):
        return None
    M = N * H * W
    dev = x.device
    out = torch.empty_like(x)
    ln2 = m2 = r2 = z = h = None
    if train:
        ln2 = torch.empty_like(x)
        m2 = torch.empty(M, device=dev, dtype=torch.float32)
        r2 = torch.empty(M, device=dev, dtype=torch.float32)
        z = torch.empty(N, H, W, Hp, device=dev, dtype=x.dtype)
        h = torch.empty(N, H, W, Hp, device=dev, dtype=x.dtype)
    flops = 2.0 * M * fc1s.cin * fc1s.cout * 2  # fc1 + fc2, unpadded
    nbytes = x.element_size() * M * (3 * Cp + ((Cp + 2 * Hp) if train else 0))
    with ktrace.span('swin_mlp_block_fwd_kernel', flops, nbytes):
        _lib.check(
            lib.sr_swin_mlp_fused_fwd(_lib.ptr(x), _lib.ptr(n2w.detach()), _lib.ptr(n2b.detach()), Creal, 1e-5,
                                      _lib.ptr(f1wf), _lib.ptr(f1bg), _lib.ptr(f2wf), _lib.ptr(f2bg), _lib.ptr(s2), N,
                                      H * W, Cp, Hp, _lib.ptr(out), _lib.ptr(ln2), _lib.ptr(m2), _lib.ptr(r2),
                                      _lib.ptr(z), _lib.ptr(h), _lib.stream()))
    return out, ln2, m2, r2, z, h


_STB_SIDE_BATCH = switch('SR_STB_SIDE_BATCH') != '0'


class _STB(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, geom, fc1s, fc2s, scale, dp, train, n1w, n1b, qw, qb, table, pw, pb, n2w, n2b, f1w, f1b, f2w,
                f2b):
        dtype = x.dtype
        N, H, W, Cp = x.shape
        Cr = geom.dim
        qwf, _, qbg = prepared_linear(qw, qb, geom.qkv, dtype)
        tab = table.detach().float().contiguous()
        pwf, _, pbg = prepared_linear(pw, pb, geom.proj, dtype)
        s1, s2 = dp if dp is not None else (None, None)  # per-sample DropPath factors (fp32 [N])
        train = train and any(ctx.needs_input_grad)  # the fused kernels store the backward's inputs only then
        fused = swin_attn_fused(x, n1w, n1b, Cr, qwf, qbg, tab, pwf, pbg, s1, geom, scale, train)
        if fused is not None:  # LN1 -> qkv -> window attention -> proj + residual in one launch
            x2, ln1, m1, r1, qkv, a, lse = fused
        else:
            fused = linear_ln_fwd(x, n1w, n1b, Cr, qwf, qbg, geom.qkv, N, H, W)  # norm1 -> qkv in one launch
            if fused is not None:
                qkv, ln1, m1, r1 = fused
            else:
                ln1, m1, r1 = layernorm(x, n1w, n1b, Cr)
                qkv = linear_fwd(ln1, qwf, qbg, geom.qkv, N, H, W)
            a, lse = window_attn(qkv, geom, N, H, W, scale, tab)
            x2 = linear_fwd(a, pwf, pbg, geom.proj, N, H, W, res=x, beta=1.0, row_scale=s1)
        f1wf, _, f1bg = prepared_linear(f1w, f1b, fc1s, dtype)
        f2wf, _, f2bg = prepared_linear(f2w, f2b, fc2s, dtype)
        fm = swin_mlp_fused(x2, n2w, n2b, Cr, f1wf, f1bg, fc1s, f2wf, f2bg, s2, train)
        if fm is not None:  # LN2 -> fc1 -> GELU -> fc2 + residual in one launch
            out, ln2, m2, r2, z, h = fm
        else:
            z = torch.empty(N, H, W, fc1s.cout_p, device=x.device, dtype=dtype)
            fused = linear_ln_fwd(x2, n2w, n2b, Cr, f1wf, f1bg, fc1s, N, H, W, act=GELU, aux=z)  # norm2 -> fc1
            if fused is not None:
                h, ln2, m2, r2 = fused
            else:
                ln2, m2, r2 = layernorm(x2, n2w, n2b, Cr)
                h = linear_fwd(ln2, f1wf, f1bg, fc1s, N, H, W, act=GELU, aux=z)
            out = linear_fwd(h, f2wf, f2bg, fc2s, N, H, W, res=x2, beta=1.0, row_scale=s2)
        ctx.geom, ctx.fc1s, ctx.fc2s, ctx.scale, ctx.dp = geom, fc1s, fc2s, scale, dp
        ctx.save_for_backward(x, ln1, m1, r1, qkv, a, lse, x2, ln2, m2, r2, z, h, tab, n1w, qw, qb, pw, pb, n2w, f1w,
                              f1b, f2w, f2b, n1b, n2b, table)
        return out

    @staticmethod
    def backward(ctx, dout):
        if _STB_SIDE_BATCH:  # the block's side-stream launches forked once, at its end (ops.conv.side_batch)
            with C.side_batch():
                return _STB._backward_body(ctx, dout)
        return _STB._backward_body(ctx, dout)

    @staticmethod
    def _backward_body(ctx, dout):
        (x, ln1, m1, r1, qkv, a, lse, x2, ln2, m2, r2, z, h, tab, n1w, qw, qb, pw, pb, n2w, f1w, f1b, f2w,
         f2b, n1b, n2b, table) = ctx.saved_tensors
        g, fc1s, fc2s, scale = ctx.geom, ctx.fc1s, ctx.fc2s, ctx.scale
        dtype = x.dtype
        N, H, W, Cp = x.shape
        Cr = g.dim
        dout = dout.to(dtype).contiguous()
        s1, s2 = ctx.dp if ctx.dp is not None else (None, None)
        g2 = row_scale(dout, s2, H * W) if s2 is not None else dout  # fc2-branch gradient
        _, f2wd, _ = prepared_linear(f2w, f2b, fc2s, dtype)
        dz = linear_dgrad(g2, f2wd, fc2s, N, H, W, gate=z, gate_mode=1)  # z: GELU' of fc1's output (its aux)
        df2w, df2b = linear_wgrad(g2, h, fc2s, N, H, W, params=(f2w, f2b))
        _, f1wd, _ = prepared_linear(f1w, f1b, fc1s, dtype)
        df1w, df1b = linear_wgrad(dz, ln2, fc1s, N, H, W, params=(f1w, f1b))
        dln2 = linear_dgrad(dz, f1wd, fc1s, N, H, W)
        dx2, dn2w, dn2b = layernorm_bwd(dln2, x2, m2, r2, n2w, Cr, res=dout, params=(n2w, n2b), row_scale=s1)
        if s1 is not None:
            dx2, g1 = dx2  # g1 = the proj-branch gradient s1 * dx2, written by the same kernel
        else:
            g1 = dx2
        _, pwd, _ = prepared_linear(pw, pb, g.proj, dtype)
        da = linear_dgrad(g1, pwd, g.proj, N, H, W)
        dpw, dpb = linear_wgrad(g1, a, g.proj, N, H, W, params=(pw, pb))
        dqkv, dtab = window_attn_bwd(qkv, a, da, lse, g, N, H, W, scale, tab, table_param=table)
        _, qwd, _ = prepared_linear(qw, qb, g.qkv, dtype)
        dqw, dqb = linear_wgrad(dqkv, ln1, g.qkv, N, H, W, params=(qw, qb))
        dln1 = linear_dgrad(dqkv, qwd, g.qkv, N, H, W)
        dx, dn1w, dn1b = layernorm_bwd(dln1, x, m1, r1, n1w, Cr, res=dx2, params=(n1w, n1b))
        return (dx, None, None, None, None, None, None, dn1w, dn1b, dqw, dqb, dtab, dpw, dpb, dn2w, dn2b, df1w, df1b, df2w,
                df2b)


def swin_block(x, blk, geom, fc1s, fc2s, dp=None):
    """dp: None, or the (s1, s2) per-sample DropPath factors of this forward."""
    at = blk.attn
    # grad mode is read here: inside Function.forward it is always off, and needs_input_grad holds under
    # torch.no_grad() too (parameters still require grad), so validation would store the backward's inputs
    return _STB.apply(x, geom, fc1s, fc2s, float(at.scale), dp, torch.is_grad_enabled(), blk.norm1.weight,
                      blk.norm1.bias, at.qkv.weight,
                      at.qkv.bias, at.relative_position_bias_table, at.proj.weight, at.proj.bias, blk.norm2.weight,
                      blk.norm2.bias, blk.mlp.fc1.weight, blk.mlp.fc1.bias, blk.mlp.fc2.weight, blk.mlp.fc2.bias)


class _AddPos(torch.autograd.Function):
    """x + absolute_pos_embed over the token map (swinir_arch.py:879-880); the embedding's gradient
    is the batch sum, accumulated straight into its flat .grad view when it has one."""

    @staticmethod
    def forward(ctx, x, pos, Creal):
        N, H, W, Cp = x.shape
        y = torch.empty_like(x)
        lib = _lib.load()
        _lib.check(lib.sr_add_pos_embed(_lib.dtype_code(x.dtype), _lib.ptr(x), N, H * W, Creal, Cp,
                                        _lib.ptr(pos.detach().contiguous()), _lib.ptr(y), _lib.stream()))
        ctx.geo = (N, H * W, Creal, Cp)
        ctx.pos = pos
        return y

    @staticmethod
    def backward(ctx, dy):
        N, P, Creal, Cp = ctx.geo
        dy = dy.contiguous()
        direct = _direct((ctx.pos, ))
        dpos = direct[0] if direct is not None else torch.empty(ctx.pos.shape, device=dy.device, dtype=torch.float32)
        lib = _lib.load()
        _lib.check(lib.sr_pos_embed_grad(_lib.dtype_code(dy.dtype), _lib.ptr(dy), N, P, Creal, Cp, _lib.ptr(dpos),
                                         int(direct is not None), _lib.stream()))
        if direct is not None:
            C.grad_ready(ctx.pos)
            return dy, None, None
        return dy, dpos, None


def add_pos_embed(x, pos, Creal):
    if x.shape[1] * x.shape[2] != pos.shape[1]:
        raise ValueError(f'absolute_pos_embed covers {pos.shape[1]} tokens, the input has {x.shape[1] * x.shape[2]} '
                         '(ape needs the runtime size to equal img_size, as in the reference)')
    return _AddPos.apply(x, pos, Creal)
