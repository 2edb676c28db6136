"""upfirdn2d on HIP (drop-in for ``basicsr.ops.upfirdn2d``).

``upfirdn2d(input, kernel, up=1, down=1, pad=(0, 0))`` of
``basicsr/ops/upfirdn2d/upfirdn2d.py:153-159``: NCHW input, 2-D FIR kernel, the same
(up, down, pad) for both axes; zero-insert upsample, pad (negative crops), convolve with
the kernel (correlation with its flip), subsample.  Backward and double-backward are the
same kernel (``sr_upfirdn2d``) on the adjoint resampling: up and down swapped, the kernel
flipped and the adjoint padding of ``_adjoint_pad`` (upfirdn2d.py:115-126).
The reference's CPU path (``upfirdn2d_native``) is restated in ``oracle/nets.py`` for the
tests; here CPU tensors raise ``NotImplementedError``.
"""
import torch
from torch.autograd import Function

from .. import _lib

__all__ = ['UpFirDn2d', 'UpFirDn2dBackward', 'upfirdn2d']


def _run(x, kernel, up_x, up_y, down_x, down_y, px0, px1, py0, py1):
    """x [major, h, w] (fp32 / bf16, contiguous) -> [major, out_h, out_w]."""
    if not x.is_cuda:
        raise NotImplementedError('upfirdn2d runs on the GPU only (HIP kernels)')
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    x = x.contiguous()
    k = kernel.detach().to(device=x.device, dtype=torch.float32).contiguous()
    major, h, w = x.shape
    kh, kw = k.shape
    oh, ow = _out_size(h, w, kh, kw, up_x, up_y, down_x, down_y, px0, px1, py0, py1)
    out = torch.empty(major, oh, ow, device=x.device, dtype=x.dtype)
    _lib.check(_lib.load().sr_upfirdn2d(_lib.dtype_code(x.dtype), _lib.ptr(x), major, h, w, _lib.ptr(k), kh, kw, up_x,
                                        up_y, down_x, down_y, px0, px1, py0, py1, _lib.ptr(out), _lib.stream()))
    return out


def _out_size(h, w, kh, kw, up_x, up_y, down_x, down_y, px0, px1, py0, py1):
    oh = (h * up_y + py0 + py1 - kh) // down_y + 1
    ow = (w * up_x + px0 + px1 - kw) // down_x + 1
    if oh <= 0 or ow <= 0:
        raise ValueError(f'upfirdn2d output would be empty ({oh}x{ow})')
    return oh, ow


def _adjoint_pad(in_h, in_w, out_h, out_w, kh, kw, up, down, pad):
    """Padding of the adjoint resampling.  Leading side: the flipped kernel's support
    mirrored (k - 1 - p0).  Trailing side: whatever makes the adjoint output exactly
    in_h x in_w after swapping the roles of up and down."""
    (up_x, up_y), (down_x, down_y), (px0, _, py0, _) = up, down, pad
    gx0, gy0 = kw - px0 - 1, kh - py0 - 1
    gx1 = in_w * up_x - out_w * down_x + px0 - up_x + 1
    gy1 = in_h * up_y - out_h * down_y + py0 - up_y + 1
    return gx0, gx1, gy0, gy1


class UpFirDn2dBackward(Function):
    """Gradient of UpFirDn2d (upfirdn2d.py:27-78); differentiable once more."""

    @staticmethod
    def forward(ctx, grad_output, kernel, grad_kernel, up, down, pad, g_pad, in_size, out_size):
        (up_x, up_y), (down_x, down_y) = up, down
        gx0, gx1, gy0, gy1 = g_pad
        g = grad_output.reshape(-1, out_size[0], out_size[1])
        gi = _run(g, grad_kernel, down_x, down_y, up_x, up_y, gx0, gx1, gy0, gy1)
        ctx.save_for_backward(kernel)
        ctx.up, ctx.down, ctx.pad, ctx.in_size, ctx.out_size = up, down, pad, in_size, out_size
        return gi.view(in_size[0], in_size[1], in_size[2], in_size[3])

    @staticmethod
    def backward(ctx, gradgrad_input):
        kernel, = ctx.saved_tensors
        (up_x, up_y), (down_x, down_y), (px0, px1, py0, py1) = ctx.up, ctx.down, ctx.pad
        gg = gradgrad_input.reshape(-1, ctx.in_size[2], ctx.in_size[3])
        out = _run(gg, kernel, up_x, up_y, down_x, down_y, px0, px1, py0, py1)
        out = out.view(ctx.in_size[0], ctx.in_size[1], ctx.out_size[0], ctx.out_size[1])
        return out, None, None, None, None, None, None, None, None


class UpFirDn2d(Function):
    """upfirdn2d.py:81-150: planes = N*C, one kernel launch."""

    @staticmethod
    def forward(ctx, input, kernel, up, down, pad):
        (up_x, up_y), (down_x, down_y), (px0, px1, py0, py1) = up, down, pad
        kh, kw = kernel.shape
        _, ch, in_h, in_w = input.shape
        out = _run(input.reshape(-1, in_h, in_w), kernel, up_x, up_y, down_x, down_y, px0, px1, py0, py1)
        out_h, out_w = out.shape[1], out.shape[2]
        ctx.save_for_backward(kernel, torch.flip(kernel, [0, 1]))
        ctx.in_size, ctx.out_size = input.shape, (out_h, out_w)
        ctx.up, ctx.down, ctx.pad = up, down, pad
        ctx.g_pad = _adjoint_pad(in_h, in_w, out_h, out_w, kh, kw, up, down, pad)
        return out.view(-1, ch, out_h, out_w)

    @staticmethod
    def backward(ctx, grad_output):
        kernel, grad_kernel = ctx.saved_tensors
        gi = UpFirDn2dBackward.apply(grad_output, kernel, grad_kernel, ctx.up, ctx.down, ctx.pad, ctx.g_pad,
                                     ctx.in_size, ctx.out_size)
        return gi, None, None, None, None


def upfirdn2d(input, kernel, up=1, down=1, pad=(0, 0)):
    """basicsr/ops/upfirdn2d/upfirdn2d.py:153-159 (GPU only: no CPU fallback)."""
    if input.device.type == 'cpu':
        raise NotImplementedError('upfirdn2d runs on the GPU only (HIP kernels)')
    return UpFirDn2d.apply(input, kernel, (up, up), (down, down), (pad[0], pad[1], pad[0], pad[1]))
