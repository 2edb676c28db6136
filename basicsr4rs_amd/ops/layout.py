"""Pixel (un)shuffle on NCHW tensors — bit-exact HIP index kernels.

Reference semantics: nn.PixelShuffle (basicsr/archs/arch_util.py:136,139) and
``pixel_unshuffle`` (basicsr/archs/arch_util.py:217-234).  Inside the nets the shuffle is
fused into the conv store / gather (csrc/conv3x3.hip); these standalone ops serve the
NCHW API and the bit-exactness tests.
"""
import torch

from .. import _lib


def _shuffle(x, r):
    N, C, H, W = x.shape
    if r > 0:
        out = (N, C // (r * r), H * r, W * r)
    else:
        s = -r
        out = (N, C * s * s, H // s, W // s)
    y = torch.empty(out, device=x.device, dtype=x.dtype)
    lib = _lib.load()
    _lib.check(lib.sr_pixel_shuffle_nchw(_lib.dtype_code(x.dtype), _lib.ptr(x), N, C, H, W, r, _lib.ptr(y),
                                         _lib.stream()))
    return y


class _PixelShuffle(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, r):
        ctx.r = r
        return _shuffle(x.contiguous(), r)

    @staticmethod
    def backward(ctx, dy):
        return _shuffle(dy.contiguous(), -ctx.r), None


def pixel_shuffle(x, upscale_factor):
    """out[n, c, h*r+i, w*r+j] = x[n, c*r*r + i*r + j, h, w]."""
    return _PixelShuffle.apply(x, int(upscale_factor))


def pixel_unshuffle(x, scale):
    """out[n, c*s*s + i*s + j, h, w] = x[n, c, h*s+i, w*s+j] (inverse of pixel_shuffle)."""
    b, c, hh, hw = x.size()
    assert hh % scale == 0 and hw % scale == 0
    return _PixelShuffle.apply(x, -int(scale))
