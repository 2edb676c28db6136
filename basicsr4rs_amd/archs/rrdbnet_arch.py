"""RRDBNet / ESRGAN generator (basicsr/archs/rrdbnet_arch.py:9-119) on the HIP engine.

Parameter names/init are the reference's; each RRDB (three dense blocks) is one fused op
(ops/blocks.py): the dense concatenations are channel slices of one buffer per block, the
residual scalings fuse into conv epilogues.  ``F.interpolate(scale_factor=2, 'nearest')``
before conv_up1/conv_up2 is folded into those convs' input gather (in_up=2).
"""
from torch import nn as nn

from .. import _lib
from ..ops import blocks as BK
from ..ops import conv as C
from ..ops.layout import pixel_unshuffle
from ..utils.registry import ARCH_REGISTRY
from .arch_util import default_init_weights, make_layer


class ResidualDenseBlock(nn.Module):
    """5 dense convs, LeakyReLU 0.2, 0.2-scaled residual (rrdbnet_arch.py:9-39)."""

    def __init__(self, num_feat=64, num_grow_ch=32):
        super().__init__()
        self.conv1 = nn.Conv2d(num_feat, num_grow_ch, 3, 1, 1)
        self.conv2 = nn.Conv2d(num_feat + num_grow_ch, num_grow_ch, 3, 1, 1)
        self.conv3 = nn.Conv2d(num_feat + 2 * num_grow_ch, num_grow_ch, 3, 1, 1)
        self.conv4 = nn.Conv2d(num_feat + 3 * num_grow_ch, num_grow_ch, 3, 1, 1)
        self.conv5 = nn.Conv2d(num_feat + 4 * num_grow_ch, num_feat, 3, 1, 1)
        self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        default_init_weights([self.conv1, self.conv2, self.conv3, self.conv4, self.conv5], 0.1)


class RRDB(nn.Module):
    """Residual in residual dense block (rrdbnet_arch.py:42-63), one fused HIP op."""

    def __init__(self, num_feat, num_grow_ch=32):
        super().__init__()
        self.rdb1 = ResidualDenseBlock(num_feat, num_grow_ch)
        self.rdb2 = ResidualDenseBlock(num_feat, num_grow_ch)
        self.rdb3 = ResidualDenseBlock(num_feat, num_grow_ch)

    def forward(self, x):
        return BK.rrdb(x, self)


@ARCH_REGISTRY.register()
class RRDBNet(nn.Module):

    def __init__(self, num_in_ch, num_out_ch, scale=4, num_feat=64, num_block=23, num_grow_ch=32):
        super().__init__()
        self.scale = scale
        self.num_out_ch = num_out_ch
        if scale == 2:
            num_in_ch = num_in_ch * 4
        elif scale == 1:
            num_in_ch = num_in_ch * 16
        self.num_in_ch = num_in_ch
        self.conv_first = nn.Conv2d(num_in_ch, num_feat, 3, 1, 1)
        self.body = make_layer(RRDB, num_block, num_feat=num_feat, num_grow_ch=num_grow_ch)
        self.conv_body = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_up1 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_up2 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_hr = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
        self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)

    def forward(self, x):
        if self.scale == 2:
            x = pixel_unshuffle(x, scale=2)
        elif self.scale == 1:
            x = pixel_unshuffle(x, scale=4)
        dt = C.feature_dtype()
        h = C.to_nhwc(x, C.pad8(self.num_in_ch), dt)
        feat = C.conv3x3(h, self.conv_first)
        feat = C.conv3x3(self.body(feat), self.conv_body, res=feat)
        lr = dict(act=_lib.ACT_LRELU, slope=0.2)
        # upsampling tail (rrdbnet_arch.py:112-119) as one chain: each lrelu backward fused into the
        # next conv's dgrad (ops/conv.py _ConvChain; RRDB x4 64.43 -> 64.29 ms, A/B 2 rounds)
        return C.conv_chain(feat, (self.conv_up1, self.conv_up2, self.conv_hr, self.conv_last),
                            (dict(in_up=2, **lr), dict(in_up=2, **lr), lr, dict(out_nchw=True)))
