"""Deformable convolution v1 / v2 on HIP (drop-in for ``basicsr.ops.dcn``).

API parity with ``basicsr/ops/dcn/deform_conv.py``: the functions ``deform_conv``
(:33-119) and ``modulated_deform_conv`` (:121-188) take the same positional arguments and
NCHW tensors, CPU tensors raise ``NotImplementedError`` (:61-62), and the four module
classes (:191-379) expose the same constructor arguments, attributes and state_dict keys
(``weight``, ``bias``, ``conv_offset.{weight,bias}``) with the same initialisation
distributions.

Execution (per call, all images at once instead of the reference's per-image loop):
  forward : x -> NHWC, ``sr_dcn_im2col`` (mask * bilinear samples as pixel-major column
            rows), 1x1 MFMA GEMM with the bias in its epilogue (``sr_conv3x3_fwd``,
            ksize 1, one call per conv group), NHWC -> NCHW; in bf16 with groups 1, 64 input
            and <= 64 output channels (EDVR's PCD / TSA shapes) one fused kernel instead
            (``sr_dcn_fwd_fused``), which stores the columns only when a backward will run.
  backward: dcols = dy x W (same GEMM on the transposed weight image), dW / db by the
            split-K wgrad kernel over (dy, cols), ``sr_dcn_col2im`` for grad x (fp32
            atomics), grad offset and grad mask in one pass; in bf16 with groups 1 and 64
            input channels (round 4) ``sr_dcn_bwd_fused`` instead of the dcols GEMM and
            col2im: each tap's dcols tile is formed on MFMA inside the coordinate-gradient and
            scatter kernels and never stored (``SR_DCN_BWD_FUSED=0`` keeps the dcols path).
Under ``torch.autocast('cuda')`` samples, columns and GEMMs run in bf16 (fp32 accumulate);
offsets, masks and all their gradients stay fp32.
"""
import math

import torch
from torch import nn
from torch.autograd import Function
from torch.autograd.function import once_differentiable
from torch.nn import functional as F
from torch.nn.modules.utils import _pair, _single

from .. import _lib
from . import conv as C
from .swin import LinearSpec
from .._switches import switch

__all__ = ['DeformConvFunction', 'ModulatedDeformConvFunction', 'deform_conv', 'modulated_deform_conv', 'DeformConv',
           'DeformConvPack', 'ModulatedDeformConv', 'ModulatedDeformConvPack', 'offset_conv', 'split_offset_mask']


def _require_gpu(*tensors):
    if any(t is not None and not t.is_cuda for t in tensors):
        raise NotImplementedError('deformable conv runs on the GPU only (HIP kernels)')


class _Geom:
    """Static geometry of one deformable conv call (shapes, padding of the GEMM operands)."""

    def __init__(self, x, weight, stride, padding, dilation, groups, deformable_groups):
        self.N, self.C, self.H, self.W = x.shape
        self.cout, cin_g, self.kh, self.kw = weight.shape
        if self.C != cin_g * groups:
            raise RuntimeError(f'Input shape and kernel channels won\'t match: ({self.C} vs {cin_g * groups}).')
        if self.C % deformable_groups:
            raise RuntimeError(f'{self.C} channels are not divisible by deformable_groups={deformable_groups}')
        (self.sh, self.sw), (self.ph, self.pw), (self.dh, self.dw) = _pair(stride), _pair(padding), _pair(dilation)
        self.G, self.DG = groups, deformable_groups
        self.Ho = (self.H + 2 * self.ph - (self.dh * (self.kh - 1) + 1)) // self.sh + 1
        self.Wo = (self.W + 2 * self.pw - (self.dw * (self.kw - 1) + 1)) // self.sw + 1
        if self.Ho <= 0 or self.Wo <= 0:
            raise ValueError(f'convolution input is too small (output would be '
                             f'{self.N}x{self.cout}x{self.Ho}x{self.Wo})')
        self.K = self.kh * self.kw
        self.cg, self.Cp = self.C // groups, C.pad8(self.C)
        self.cgp = C.pad8(self.cg)
        self.cout_g = self.cout // groups
        if groups > 1 and self.cout_g % 8:
            raise NotImplementedError('grouped deformable conv needs out_channels / groups to be a multiple of 8')
        self.cout_gp = C.pad8(self.cout_g)
        self.L = groups * self.K * self.cgp  # column row length
        self.ldy = groups * self.cout_gp

    def desc(self, dtype):
        d = _lib.DcnDesc()
        d.dtype = _lib.dtype_code(dtype)
        d.N, d.C, d.H, d.W, d.Cp, d.Ho, d.Wo = self.N, self.C, self.H, self.W, self.Cp, self.Ho, self.Wo
        d.kh, d.kw, d.stride_h, d.stride_w = self.kh, self.kw, self.sh, self.sw
        d.pad_h, d.pad_w, d.dil_h, d.dil_w = self.ph, self.pw, self.dh, self.dw
        d.groups, d.deformable_groups, d.cgp = self.G, self.DG, self.cgp
        return d

    def spec(self):
        # GEMM column k = tap * cgp + ci  <->  parameter column ci * K + tap (weight.flatten(1))
        K, cg, cgp = self.K, self.cg, self.cgp
        col_map = [(ci * K + tap) if ci < cg else -1 for tap in range(K) for ci in range(cgp)]
        return LinearSpec(cg * K, self.cout_g, K * cgp, self.cout_gp, None, col_map)


_SPECS = {}


def _spec(g):
    key = (g.C, g.cout, g.kh, g.kw, g.G)
    if key not in _SPECS:
        _SPECS[key] = g.spec()
    return _SPECS[key]


def _prepared(weight, bias, g, spec, dtype):
    """GEMM images (wf [cout_gp][K*cgp], wd [K*cgp][cout_gp], bias) per conv group, cached."""
    key = (weight._version, C._PARAM_EPOCH[0], dtype, weight.data_ptr(), -1 if bias is None else bias._version)
    cache = getattr(weight, '_sr_dcn_prep', None)
    if cache is not None and cache[0] == key:
        return cache[1]
    dev = weight.device
    rm, cm, _, _ = spec.maps(dev)
    lib = _lib.load()
    w = weight.detach().contiguous()
    images = []
    for gi in range(g.G):
        rows = slice(gi * g.cout_g, (gi + 1) * g.cout_g)
        wg = w[rows]
        bgi = bias.detach()[rows].contiguous() if bias is not None else None
        wf = torch.empty(spec.cout_p, spec.cin_p, device=dev, dtype=dtype)
        wd = torch.empty(spec.cin_p, spec.cout_p, device=dev, dtype=dtype)
        bg = torch.empty(spec.cout_p, device=dev, dtype=torch.float32)
        _lib.check(
            lib.sr_conv_prep_mapped(_lib.dtype_code(dtype), 1, _lib.ptr(wg), _lib.ptr(bgi), spec.cout, spec.cin,
                                    spec.cout_p, spec.cin_p, 0, _lib.ptr(rm), _lib.ptr(cm), _lib.ptr(wf),
                                    _lib.ptr(wd), _lib.ptr(bg), _lib.stream()))
        images.append((wf, wd, bg))
    weight._sr_dcn_prep = (key, images)
    return images


def fused_ok(g, dtype):
    """True when the forward runs as one kernel (``sr_dcn_fwd_fused``: bf16, groups 1, 64 input
    channels, <= 64 outputs; the column matrix is built per tap in LDS and not stored unless the
    backward needs it)."""
    return dtype == torch.bfloat16 and bool(_lib.load().sr_dcn_fwd_fused_ok(g.desc(dtype), g.cout))


def _dcn_forward(x, offset, mask, weight, bias, g, dtype, need_cols=True):
    lib = _lib.load()
    off = offset.float().contiguous()
    msk = None if mask is None else mask.float().contiguous()
    if tuple(off.shape) != (g.N, g.DG * 2 * g.K, g.Ho, g.Wo):
        raise RuntimeError(f'offset shape {tuple(off.shape)} != {(g.N, g.DG * 2 * g.K, g.Ho, g.Wo)}')
    if msk is not None and tuple(msk.shape) != (g.N, g.DG * g.K, g.Ho, g.Wo):
        raise RuntimeError(f'mask shape {tuple(msk.shape)} != {(g.N, g.DG * g.K, g.Ho, g.Wo)}')
    if fused_ok(g, dtype):
        xh = C.nchw_to_nhwc(x.float(), g.Cp, dtype)
        wf, _, bg = _prepared(weight, bias, g, _spec(g), dtype)[0]
        y = torch.empty(g.N, g.cout, g.Ho, g.Wo, device=x.device, dtype=torch.float32)
        cols = torch.empty(g.N, g.Ho, g.Wo, g.L, device=x.device, dtype=dtype) if need_cols else None
        _lib.check(lib.sr_dcn_fwd_fused(g.desc(dtype), _lib.ptr(xh), 0, _lib.ptr(off), _lib.ptr(msk), _lib.ptr(wf),
                                        wf.shape[1], wf.shape[0], g.cout, _lib.ptr(bg if bias is not None else None),
                                        _lib.ptr(y), _lib.ptr(cols), _lib.stream()))
        return y, (xh, off, msk, cols)
    xh = C.nchw_to_nhwc(x.float(), g.Cp, dtype)
    cols = torch.empty(g.N, g.Ho, g.Wo, g.L, device=x.device, dtype=dtype)
    _lib.check(lib.sr_dcn_im2col(g.desc(dtype), _lib.ptr(xh), _lib.ptr(off), _lib.ptr(msk), _lib.ptr(cols),
                                 _lib.stream()))
    images = _prepared(weight, bias, g, _spec(g), dtype)
    y = torch.empty(g.N, g.Ho, g.Wo, g.ldy, device=x.device, dtype=dtype)
    kc = g.K * g.cgp
    for gi, (wf, _, bg) in enumerate(images):
        C.conv_fwd_raw(cols, wf, None if bias is None else bg, y, g.N, g.Ho, g.Wo, kc, g.cout_gp, g.cout_gp,
                       ksize=1, ldx=g.L, xcoff=gi * kc, ldy=g.ldy, ycoff=gi * g.cout_gp)
    return C.nhwc_to_nchw(y, g.cout), (xh, off, msk, cols)


BWD_FUSED = switch('SR_DCN_BWD_FUSED') != '0'


def bwd_fused_ok(g, dtype):
    """True when the backward runs without the dcols matrix (``sr_dcn_bwd_fused``: bf16, groups 1,
    64 input channels, <= 64 outputs)."""
    return (BWD_FUSED and dtype == torch.bfloat16 and g.G == 1
            and bool(_lib.load().sr_dcn_bwd_fused_ok(g.desc(dtype), g.cout_gp)))


def _dcn_backward(grad_out, saved, weight, bias, g, dtype):
    xh, off, msk, cols = saved
    lib = _lib.load()
    spec = _spec(g)
    images = _prepared(weight, bias, g, spec, dtype)
    dyh = C.nchw_to_nhwc(grad_out.float(), g.ldy, dtype)
    fused = bwd_fused_ok(g, dtype)
    dcols = None if fused else torch.empty(g.N, g.Ho, g.Wo, g.L, device=dyh.device, dtype=dtype)
    ci_map = spec.maps(dyh.device)[3]
    kc = g.K * g.cgp
    dws, dbs = [], []
    for gi, (_, wd, _) in enumerate(images):
        if not fused:
            C.conv_fwd_raw(dyh, wd, None, dcols, g.N, g.Ho, g.Wo, g.cout_gp, kc, kc, ksize=1, ldx=g.ldy,
                           xcoff=gi * g.cout_gp, ldy=g.L, ycoff=gi * kc)
        dw, db = C.conv_wgrad_raw(dyh, cols, g.N, g.Ho, g.Wo, kc, g.cg * g.K, g.cout_gp, g.cout_g, ksize=1,
                                  ci_map=ci_map, ldx=g.L, xcoff=gi * kc, ldy=g.ldy, ycoff=gi * g.cout_gp,
                                  need_bias=bias is not None)
        dws.append(dw.reshape(g.cout_g, g.cg, g.kh, g.kw))
        dbs.append(db)
    grad_weight = torch.cat(dws, 0) if g.G > 1 else dws[0]
    grad_bias = None if bias is None else (torch.cat(dbs, 0) if g.G > 1 else dbs[0])
    goff = torch.empty_like(off)
    gmask = None if msk is None else torch.empty_like(msk)
    d = g.desc(dtype)
    wsb = lib.sr_dcn_col2im_workspace(d)
    ws = torch.empty(wsb // 4 + 1, device=dyh.device, dtype=torch.int32)
    if fused:  # grad x written in full, NCHW
        wd = images[0][1]
        gx = torch.empty(g.N, g.C, g.H, g.W, device=dyh.device, dtype=torch.float32)
        _lib.check(
            lib.sr_dcn_bwd_fused(d, _lib.ptr(dyh), g.ldy, _lib.ptr(wd), wd.shape[1], g.cout_gp, _lib.ptr(xh),
                                 _lib.ptr(off), _lib.ptr(msk), _lib.ptr(gx), 1, _lib.ptr(goff), _lib.ptr(gmask),
                                 _lib.ptr(ws), wsb, _lib.stream()))
        return gx, goff, gmask, grad_weight, grad_bias
    gx = torch.zeros(g.N, g.H, g.W, g.Cp, device=dyh.device, dtype=torch.float32)
    _lib.check(
        lib.sr_dcn_col2im(d, _lib.ptr(dcols), _lib.ptr(xh), _lib.ptr(off), _lib.ptr(msk), _lib.ptr(gx),
                          _lib.ptr(goff), _lib.ptr(gmask), _lib.ptr(ws), wsb, _lib.stream()))
    return C.nhwc_to_nchw(gx, g.C), goff, gmask, grad_weight, grad_bias


def _save(ctx, g, dtype, x, saved, weight, bias):
    ctx.g, ctx.dtype, ctx.in_dtype = g, dtype, x.dtype
    ctx.has_mask = saved[2] is not None
    xh, off, msk, cols = saved
    ctx.save_for_backward(xh, off, msk if msk is not None else off.new_empty(0), cols, weight,
                          bias if bias is not None else off.new_empty(0))
    ctx.has_bias = bias is not None


def _restore(ctx):
    xh, off, msk, cols, weight, bias = ctx.saved_tensors
    return (xh, off, msk if ctx.has_mask else None, cols), weight, (bias if ctx.has_bias else None)


class DeformConvFunction(Function):
    """DCNv1 (basicsr/ops/dcn/deform_conv.py:33-119); ``im2col_step`` is validated like the
    reference but every image is processed in one batched launch."""

    @staticmethod
    def forward(ctx, input, offset, weight, stride=1, padding=0, dilation=1, groups=1, deformable_groups=1,
                im2col_step=64):
        if input is not None and input.dim() != 4:
            raise ValueError(f'Expected 4D tensor as input, got {input.dim()}D tensor instead.')
        _require_gpu(input, offset, weight)
        step = min(im2col_step, input.shape[0])
        if input.shape[0] % step:
            raise AssertionError('im2col step must divide batchsize')
        dtype = C.feature_dtype()
        g = _Geom(input, weight, stride, padding, dilation, groups, deformable_groups)
        out, saved = _dcn_forward(input, offset, None, weight, None, g, dtype, _GRAD[0] and any(ctx.needs_input_grad))
        _save(ctx, g, dtype, input, saved, weight, None)
        return out.to(input.dtype)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        _require_gpu(grad_output)
        saved, weight, _ = _restore(ctx)
        gx, goff, _, gw, _ = _dcn_backward(grad_output, saved, weight, None, ctx.g, ctx.dtype)
        need = ctx.needs_input_grad
        return (gx.to(ctx.in_dtype) if need[0] else None, goff if need[1] else None, gw if need[2] else None,
                None, None, None, None, None)


class ModulatedDeformConvFunction(Function):
    """DCNv2 (basicsr/ops/dcn/deform_conv.py:121-188)."""

    @staticmethod
    def forward(ctx, input, offset, mask, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                deformable_groups=1):
        _require_gpu(input, offset, mask, weight)
        dtype = C.feature_dtype()
        g = _Geom(input, weight, stride, padding, dilation, groups, deformable_groups)
        out, saved = _dcn_forward(input, offset, mask, weight, bias, g, dtype, _GRAD[0] and any(ctx.needs_input_grad))
        _save(ctx, g, dtype, input, saved, weight, bias)
        return out.to(input.dtype)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        _require_gpu(grad_output)
        saved, weight, bias = _restore(ctx)
        gx, goff, gmask, gw, gb = _dcn_backward(grad_output, saved, weight, bias, ctx.g, ctx.dtype)
        return (gx.to(ctx.in_dtype), goff, gmask, gw, gb, None, None, None, None, None)


# Grad mode at the call: inside Function.forward it is always off, and needs_input_grad holds under
# torch.no_grad() too (weights still require grad), so an inference call would store the columns.
_GRAD = [True]


def _with_grad_mode(fn):
    def call(*args):
        prev, _GRAD[0] = _GRAD[0], torch.is_grad_enabled()
        try:
            return fn(*args)
        finally:
            _GRAD[0] = prev
    call.__name__ = fn.__name__ if hasattr(fn, '__name__') else 'apply'
    return call


deform_conv = _with_grad_mode(DeformConvFunction.apply)
modulated_deform_conv = _with_grad_mode(ModulatedDeformConvFunction.apply)


def _offset_conv(conv, x):
    """Offset/mask branch (an nn.Conv2d) on HIP: the implicit-GEMM 3x3 conv for 3x3 / stride 1 /
    pad 1, any other geometry as a deformable conv with zero offsets and unit masks (bilinear
    sampling at integer tap positions is exact, and the reference's validity rule
    -1 < h < H gives exactly the zero padding)."""
    std = (conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
           and conv.dilation == (1, 1) and conv.groups == 1)
    if std:
        xh = C.to_nhwc(x, C.pad8(conv.in_channels), C.feature_dtype())
        return C.to_nchw(C.conv3x3(xh, conv), conv.out_channels)
    if conv.padding_mode != 'zeros' or isinstance(conv.padding, str):
        raise NotImplementedError('offset conv: only numeric zero padding is on the HIP path')
    g = _Geom(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups, 1)
    off = torch.zeros(g.N, 2 * g.K, g.Ho, g.Wo, device=x.device, dtype=torch.float32)
    msk = torch.ones(g.N, g.K, g.Ho, g.Wo, device=x.device, dtype=torch.float32)
    return modulated_deform_conv(x, off, msk, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation,
                                 conv.groups, 1)


class _DeformBase(nn.Module):
    """Shared parameters / geometry of the four deformable conv modules.

    ``pair_geometry`` keeps stride/padding/dilation as 2-tuples (DeformConv) or as given
    (ModulatedDeformConv, whose reference stores the raw ints)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding, dilation, groups,
                 deformable_groups, bias, pair_geometry):
        super().__init__()
        geom = (lambda v: _pair(v)) if pair_geometry else (lambda v: v)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride, self.padding, self.dilation = geom(stride), geom(padding), geom(dilation)
        self.groups, self.deformable_groups = groups, deformable_groups
        self.transposed, self.output_padding = False, _single(0)
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels // groups, *self.kernel_size))
        self.register_parameter('bias', nn.Parameter(torch.empty(out_channels)) if bias else None)

    def _uniform_weight(self):
        # U(-1/sqrt(fan), 1/sqrt(fan)) with fan = in_channels * kh * kw (deform_conv.py:223-228)
        bound = 1.0 / math.sqrt(self.in_channels * self.kernel_size[0] * self.kernel_size[1])
        self.weight.data.uniform_(-bound, bound)

    def _make_offset_conv(self, per_tap):
        k = self.kernel_size
        self.conv_offset = nn.Conv2d(self.in_channels, self.deformable_groups * per_tap * k[0] * k[1], k,
                                     _pair(self.stride), _pair(self.padding), _pair(self.dilation), bias=True)
        self.conv_offset.weight.data.zero_()
        self.conv_offset.bias.data.zero_()


class DeformConv(_DeformBase):
    """basicsr/ops/dcn/deform_conv.py:191-241: DCNv1, no bias; inputs smaller than the kernel
    are zero-padded bottom/right and the output cropped back."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 deformable_groups=1, bias=False):
        if bias:
            raise AssertionError('DeformConv has no bias')
        if in_channels % groups or out_channels % groups:
            raise AssertionError(f'in_channels {in_channels} / out_channels {out_channels} '
                                 f'are not divisible by groups {groups}')
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, deformable_groups,
                         False, True)
        self.reset_parameters()

    def reset_parameters(self):
        self._uniform_weight()

    def forward(self, x, offset):
        kh, kw = self.kernel_size
        ph, pw = max(kh - x.size(2), 0), max(kw - x.size(3), 0)
        if ph or pw:
            x = F.pad(x, (0, pw, 0, ph)).contiguous()
            offset = F.pad(offset, (0, pw, 0, ph)).contiguous()
        out = deform_conv(x, offset, self.weight, self.stride, self.padding, self.dilation, self.groups,
                          self.deformable_groups)
        if ph or pw:
            out = out[:, :, :out.size(2) - ph, :out.size(3) - pw].contiguous()
        return out


class DeformConvPack(DeformConv):
    """basicsr/ops/dcn/deform_conv.py:244-286: offsets predicted from the input by a
    zero-initialised conv (``conv_offset``)."""

    _version = 2

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._make_offset_conv(2)

    def init_offset(self):
        self.conv_offset.weight.data.zero_()
        self.conv_offset.bias.data.zero_()

    def forward(self, x):
        return deform_conv(x, _offset_conv(self.conv_offset, x), self.weight, self.stride, self.padding,
                           self.dilation, self.groups, self.deformable_groups)


class ModulatedDeformConv(_DeformBase):
    """basicsr/ops/dcn/deform_conv.py:289-333: DCNv2 with explicit offset and mask."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 deformable_groups=1, bias=True):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, deformable_groups,
                         bias, False)
        self.with_bias = bias
        self.init_weights()

    def init_weights(self):
        self._uniform_weight()
        if self.bias is not None:
            self.bias.data.zero_()

    def forward(self, x, offset, mask):
        return modulated_deform_conv(x, offset, mask, self.weight, self.bias, self.stride, self.padding,
                                     self.dilation, self.groups, self.deformable_groups)


def split_offset_mask(out):
    """[o1 | o2 | m] channel thirds -> offset cat(o1, o2), sigmoid mask (deform_conv.py:372-375)."""
    o1, o2, m = torch.chunk(out, 3, dim=1)
    return torch.cat((o1, o2), dim=1), torch.sigmoid(m)


class ModulatedDeformConvPack(ModulatedDeformConv):
    """basicsr/ops/dcn/deform_conv.py:336-379: offsets and sigmoid masks predicted from the
    input by a zero-initialised conv."""

    _version = 2

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._make_offset_conv(3)
        self.init_weights()  # the reference re-draws `weight` after building conv_offset (same RNG stream)

    def init_weights(self):
        super().init_weights()
        if hasattr(self, 'conv_offset'):
            self.conv_offset.weight.data.zero_()
            self.conv_offset.bias.data.zero_()

    def forward(self, x):
        offset, mask = split_offset_mask(_offset_conv(self.conv_offset, x))
        return modulated_deform_conv(x, offset, mask, self.weight, self.bias, self.stride, self.padding,
                                     self.dilation, self.groups, self.deformable_groups)


offset_conv = _offset_conv
