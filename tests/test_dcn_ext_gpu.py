"""The ``deform_conv_ext`` drop-in (ops/deform_conv_ext.py -> csrc/dcn_ext.hip) driven the way the
reference's autograd Functions drive their pybind extension (basicsr/ops/dcn/deform_conv.py:33-188):
caller-allocated output / zeroed grads / empty ``columns`` and ``ones`` buffers, the same positional
arguments (kW before kH, stride / padding / dilation as (w, h) pairs for v1, scalars for v2,
``im2col_step`` = min(step, N), ``scale`` 1), against the float64 numpy oracle (oracle/ops.py).

Also: the op config of BASELINE C5 (x [N, 64, 128, 128], deformable_groups 8; N reduced to 1), the
v1 im2col_step chunking, and the accumulate semantics of the parameter gradient (+= scale * dW)."""
import numpy as np
import pytest
import torch
from torch.autograd import Function

from basicsr4rs_amd.ops import deform_conv_ext
from oracle import ops as O
from tests.test_ops_gpu import DCN_CASES, _dcn_inputs, rel

pytestmark = pytest.mark.gpu


def _p(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class _V1(Function):
    """The reference's DeformConvFunction call sequence over ``deform_conv_ext``."""

    @staticmethod
    def forward(ctx, x, offset, weight, stride, padding, dilation, groups, dg, im2col_step):
        ctx.geo = (_p(stride), _p(padding), _p(dilation), groups, dg, im2col_step)
        ctx.save_for_backward(x, offset, weight)
        (sh, sw), (ph, pw), (dh, dw) = ctx.geo[:3]
        kh, kw = weight.shape[2:]
        Ho = (x.shape[2] + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
        Wo = (x.shape[3] + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
        out = x.new_empty(x.shape[0], weight.shape[0], Ho, Wo)
        ctx.bufs = [x.new_empty(0), x.new_empty(0)]
        step = min(im2col_step, x.shape[0])
        assert x.shape[0] % step == 0
        r = deform_conv_ext.deform_conv_forward(x, weight, offset, out, ctx.bufs[0], ctx.bufs[1], kw, kh, sw, sh, pw, ph,
                                                dw, dh, groups, dg, step)
        assert r == 1
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, offset, weight = ctx.saved_tensors
        (sh, sw), (ph, pw), (dh, dw), groups, dg, im2col_step = ctx.geo
        kh, kw = weight.shape[2:]
        step = min(im2col_step, x.shape[0])
        gx, goff = torch.zeros_like(x), torch.zeros_like(offset)
        deform_conv_ext.deform_conv_backward_input(x, offset, grad_out, gx, goff, weight, ctx.bufs[0], kw, kh, sw, sh,
                                                   pw, ph, dw, dh, groups, dg, step)
        gw = torch.zeros_like(weight)
        deform_conv_ext.deform_conv_backward_parameters(x, offset, grad_out, gw, ctx.bufs[0], ctx.bufs[1], kw, kh, sw,
                                                        sh, pw, ph, dw, dh, groups, dg, 1, step)
        return gx, goff, gw, None, None, None, None, None, None


class _V2(Function):
    """The reference's ModulatedDeformConvFunction call sequence over ``deform_conv_ext``."""

    @staticmethod
    def forward(ctx, x, offset, mask, weight, bias, stride, padding, dilation, groups, dg):
        ctx.geo = (stride, padding, dilation, groups, dg)
        ctx.with_bias = bias is not None
        if not ctx.with_bias:
            bias = x.new_empty(1)
        ctx.save_for_backward(x, offset, mask, weight, bias)
        kh, kw = weight.shape[2:]
        Ho = (x.shape[2] + 2 * padding - (dilation * (kh - 1) + 1)) // stride + 1
        Wo = (x.shape[3] + 2 * padding - (dilation * (kw - 1) + 1)) // stride + 1
        out = x.new_empty(x.shape[0], weight.shape[0], Ho, Wo)
        ctx.bufs = [x.new_empty(0), x.new_empty(0)]
        deform_conv_ext.modulated_deform_conv_forward(x, weight, bias, ctx.bufs[0], offset, mask, out, ctx.bufs[1], kh, kw,
                                                      stride, stride, padding, padding, dilation, dilation, groups, dg,
                                                      ctx.with_bias)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, offset, mask, weight, bias = ctx.saved_tensors
        stride, padding, dilation, groups, dg = ctx.geo
        kh, kw = weight.shape[2:]
        gx, goff, gm = torch.zeros_like(x), torch.zeros_like(offset), torch.zeros_like(mask)
        gw, gb = torch.zeros_like(weight), torch.zeros_like(bias)
        deform_conv_ext.modulated_deform_conv_backward(x, weight, bias, ctx.bufs[0], offset, mask, ctx.bufs[1], gx, gw, gb,
                                                       goff, gm, grad_out, kh, kw, stride, stride, padding, padding,
                                                       dilation, dilation, groups, dg, ctx.with_bias)
        return gx, goff, gm, gw, (gb if ctx.with_bias else None), None, None, None, None, None


OP_CONFIG = (1, 64, 128, 128, 64, 3, 1, 1, 1, 1, 8, True)  # C5 DCNv2 op (EDVR PCD), N reduced to 1


@pytest.mark.parametrize('case', DCN_CASES + [OP_CONFIG])
def test_deform_conv_ext_matches_oracle(cuda, case):
    N, C, H, W, Cout, k, s, p, d, groups, dg, modulated = case
    x, off, msk, w, b, dy = _dcn_inputs(case)
    t = [torch.tensor(a, device=cuda, requires_grad=True) if a is not None else None for a in (x, off, msk, w, b)]
    if modulated:
        out = _V2.apply(t[0], t[1], t[2], t[3], t[4], s, p, d, groups, dg)
    else:
        out = _V1.apply(t[0], t[1], t[3], s, p, d, groups, dg, 64)
    ref = O.dcn_forward(x, off, msk, w, b, s, p, d, groups, dg)
    assert out.shape == ref.shape
    assert rel(out, ref) < 1e-4, rel(out, ref)
    out.backward(torch.tensor(dy, device=cuda))
    grads = O.dcn_backward(x, off, msk, w, b, s, p, d, groups, dg, dy)
    for name, g, tt in zip(('x', 'offset', 'mask', 'weight', 'bias'), grads, t):
        if tt is None:
            continue
        assert rel(tt.grad, g) < 1e-4, (name, rel(tt.grad, g))


def test_deform_conv_ext_im2col_step_and_accumulate(cuda):
    """v1 with im2col_step 2 over N 4 (two chunks) equals the whole-batch result; the parameter
    gradient accumulates (+= scale * dW) and grad_input accumulates into the caller's buffer."""
    case = (4, 16, 9, 9, 24, 3, 1, 1, 1, 1, 2, False)
    x, off, _, w, _, dy = _dcn_inputs(case, seed=3)
    X, OFF, Wt, DY = (torch.tensor(a, device=cuda) for a in (x, off, w, dy))
    e = X.new_empty(0)
    outs = []
    for step in (2, 4):
        o = X.new_empty(4, 24, 9, 9)
        deform_conv_ext.deform_conv_forward(X, Wt, OFF, o, e, e, 3, 3, 1, 1, 1, 1, 1, 1, 1, 2, step)
        outs.append(o)
    assert torch.allclose(outs[0], outs[1], atol=1e-6)
    assert rel(outs[0], O.dcn_forward(x, off, None, w, None, 1, 1, 1, 1, 2)) < 1e-4
    gx_ref, goff_ref, _, gw_ref, _ = O.dcn_backward(x, off, None, w, None, 1, 1, 1, 1, 2, dy)
    gw = torch.ones_like(Wt)
    deform_conv_ext.deform_conv_backward_parameters(X, OFF, DY, gw, e, e, 3, 3, 1, 1, 1, 1, 1, 1, 1, 2, 0.5, 2)
    assert rel(gw, 1.0 + 0.5 * gw_ref) < 1e-4
    gx = torch.full_like(X, 2.0)
    goff = torch.zeros_like(OFF)
    deform_conv_ext.deform_conv_backward_input(X, OFF, DY, gx, goff, Wt, e, 3, 3, 1, 1, 1, 1, 1, 1, 1, 2, 2)
    assert rel(gx, 2.0 + gx_ref) < 1e-4 and rel(goff, goff_ref) < 1e-4


def test_deform_conv_ext_errors(cuda):
    x = torch.zeros(3, 8, 6, 6, device=cuda)
    w = torch.zeros(8, 8, 3, 3, device=cuda)
    off = torch.zeros(3, 18, 6, 6, device=cuda)
    out = torch.empty(3, 8, 6, 6, device=cuda)
    e = x.new_empty(0)
    with pytest.raises(RuntimeError, match='im2col step'):
        deform_conv_ext.deform_conv_forward(x, w, off, out, e, e, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 2)
    with pytest.raises(NotImplementedError):
        deform_conv_ext.deform_conv_forward(x.cpu(), w, off, out, e, e, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1)
    with pytest.raises(RuntimeError, match='float32'):
        deform_conv_ext.deform_conv_forward(x.double(), w, off, out, e, e, 3, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1)


def test_dcnv2pack_matches_oracle_and_warns(cuda):
    """DCNv2Pack (arch_util.py:237-263): offsets / masks from a second feature, the HIP DCNv2 path,
    and the 'Offset abs mean ... larger than 50' warning."""
    import logging

    import torch.nn.functional as F

    from basicsr4rs_amd.archs.arch_util import DCNv2Pack
    torch.manual_seed(0)
    m = DCNv2Pack(16, 24, 3, stride=1, padding=1, deformable_groups=2)
    with torch.no_grad():
        m.conv_offset.weight.normal_(0, 0.05)
        m.conv_offset.bias.normal_(0, 0.5)
        m.bias.normal_()
    x = torch.randn(2, 16, 10, 9)
    feat = torch.randn(2, 16, 10, 9)
    with torch.no_grad():
        o = F.conv2d(feat.double(), m.conv_offset.weight.double(), m.conv_offset.bias.double(), padding=1)
    o1, o2, mk = torch.chunk(o, 3, dim=1)
    off, msk = torch.cat((o1, o2), 1).numpy(), torch.sigmoid(mk).numpy()
    ref = O.dcn_forward(x.numpy(), off, msk, m.weight.detach().numpy(), m.bias.detach().numpy(), 1, 1, 1, 1, 2)
    g = m.to(cuda)
    out = g(x.to(cuda), feat.to(cuda))
    assert rel(out, ref) < 1e-4, rel(out, ref)
    records = []
    h = logging.Handler()
    h.emit = records.append
    logging.getLogger('basicsr').addHandler(h)
    try:
        with torch.no_grad():
            g.conv_offset.bias.fill_(80.0)
        g(x.to(cuda), feat.to(cuda))
    finally:
        logging.getLogger('basicsr').removeHandler(h)
    assert any('larger than 50' in r.getMessage() for r in records)


def test_offset_conv_general_geometry_on_hip(cuda):
    """A DeformConvPack whose offset conv is not 3x3 / stride 1 / pad 1 (here stride 2, pad 1, with
    the main conv strided alike) runs its offset branch on the HIP DCN path (zero offsets, unit
    masks), matching a plain float64 conv + the oracle."""
    import torch.nn.functional as F

    from basicsr4rs_amd.ops.dcn import DeformConvPack
    torch.manual_seed(1)
    m = DeformConvPack(8, 16, 3, stride=2, padding=1)
    with torch.no_grad():
        m.conv_offset.weight.normal_(0, 0.1)
        m.conv_offset.bias.normal_(0, 0.3)
    x = torch.randn(2, 8, 11, 12)
    with torch.no_grad():
        off = F.conv2d(x.double(), m.conv_offset.weight.double(), m.conv_offset.bias.double(), stride=2, padding=1)
    ref = O.dcn_forward(x.numpy(), off.numpy(), None, m.weight.detach().numpy(), None, 2, 1, 1, 1, 1)
    out = m.to(cuda)(x.to(cuda))
    assert rel(out, ref) < 1e-4, rel(out, ref)
