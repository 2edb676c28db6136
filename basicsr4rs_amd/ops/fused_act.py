"""fused_leaky_relu on the HIP engine (basicsr/ops/fused_act/fused_act.py:30-95).

Same Python surface as the reference op: ``fused_bias_act`` (the pybind entry
``fused_act_ext.fused_bias_act(input, bias, refer, act, grad, alpha, scale)``,
basicsr/ops/fused_act/src/fused_bias_act.cpp:14-26: callee allocates, input made contiguous),
the autograd Functions ``FusedLeakyReLUFunction`` / ``FusedLeakyReLUFunctionBackward`` (first
and second derivatives), the ``FusedLeakyReLU`` module (bias parameter ``bias``, zero-init) and
``fused_leaky_relu(input, bias, negative_slope=0.2, scale=2**0.5)``.

Arithmetic (fused_bias_act_kernel.cu:19-50): y = scale * lrelu(x + b[c], alpha) with the bias
broadcast on dim 1; backward dx = dy * scale * (out > 0 ? 1 : alpha) — computed here together
with the bias gradient (the reference's separate ``grad_input.sum(dim)``) in one HIP pass
(sr_fused_lrelu_bwd); double backward through ``fused_bias_act(gg, gb, out, 3, 1, ...)``.
"""
import torch
from torch import nn
from torch.autograd import Function

from .. import _lib


def _rcs(t):
    R = t.shape[0]
    C = t.shape[1] if t.dim() > 1 else 1
    S = 1
    for s in t.shape[2:]:
        S *= s
    return R, C, S


def fused_bias_act(input, bias, refer, act, grad, alpha, scale):
    """out = scale * act(input + bias) (grad=0), or the first / second derivative modes
    (grad=1, 2) gated by ``refer`` -- fused_act_ext.fused_bias_act."""
    x = input.contiguous()
    if x.dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError(f'fused_bias_act: dtype {x.dtype} not supported (float32 / bfloat16)')
    b = bias.contiguous().to(x.dtype) if bias is not None and bias.numel() > 0 else None
    r = refer.contiguous().to(x.dtype) if refer is not None and refer.numel() > 0 else None
    out = torch.empty_like(x)
    _, C, S = _rcs(x) if x.dim() >= 1 else (1, 1, 1)
    lib = _lib.load()
    _lib.check(
        lib.sr_fused_bias_act(_lib.dtype_code(x.dtype), _lib.ptr(x), _lib.ptr(b), _lib.ptr(r), _lib.ptr(out),
                              x.numel(), S, b.numel() if b is not None else 0, int(act), int(grad), float(alpha),
                              float(scale), _lib.stream()))
    return out


class FusedLeakyReLUFunctionBackward(Function):
    """(grad_output, out) -> (grad_input, grad_bias); differentiable once more."""

    @staticmethod
    def forward(ctx, grad_output, out, negative_slope, scale):
        ctx.save_for_backward(out)
        ctx.negative_slope, ctx.scale = negative_slope, scale
        dy = grad_output.contiguous()
        R, C, S = _rcs(dy)
        dx = torch.empty_like(dy)
        db = torch.empty(C, device=dy.device, dtype=torch.float32)
        lib = _lib.load()
        wsb = lib.sr_fused_lrelu_bwd_workspace(R, C, S)
        ws = torch.empty(max(1, wsb // 4 + 1), device=dy.device, dtype=torch.float32)
        _lib.check(
            lib.sr_fused_lrelu_bwd(_lib.dtype_code(dy.dtype), _lib.ptr(dy), _lib.ptr(out.contiguous()), _lib.ptr(dx),
                                   _lib.ptr(db), R, C, S, float(negative_slope), float(scale), _lib.ptr(ws), wsb,
                                   _lib.stream()))
        return dx, db.to(dy.dtype)

    @staticmethod
    def backward(ctx, gradgrad_input, gradgrad_bias):
        out, = ctx.saved_tensors
        gg = fused_bias_act(gradgrad_input, gradgrad_bias, out, 3, 1, ctx.negative_slope, ctx.scale)
        return gg, None, None, None


class FusedLeakyReLUFunction(Function):

    @staticmethod
    def forward(ctx, input, bias, negative_slope, scale):
        out = fused_bias_act(input, bias, None, 3, 0, negative_slope, scale)
        ctx.save_for_backward(out)
        ctx.negative_slope, ctx.scale = negative_slope, scale
        return out

    @staticmethod
    def backward(ctx, grad_output):
        out, = ctx.saved_tensors
        gi, gb = FusedLeakyReLUFunctionBackward.apply(grad_output, out, ctx.negative_slope, ctx.scale)
        return gi, gb, None, None


class FusedLeakyReLU(nn.Module):
    """Bias + LeakyReLU(negative_slope) * scale (basicsr/ops/fused_act/fused_act.py:76-88)."""

    def __init__(self, channel, negative_slope=0.2, scale=2**0.5):
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(channel))
        self.negative_slope = negative_slope
        self.scale = scale

    def forward(self, input):
        return fused_leaky_relu(input, self.bias, self.negative_slope, self.scale)


def fused_leaky_relu(input, bias, negative_slope=0.2, scale=2**0.5):
    return FusedLeakyReLUFunction.apply(input, bias, negative_slope, scale)
