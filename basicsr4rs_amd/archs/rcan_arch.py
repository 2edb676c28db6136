"""RCAN (basicsr/archs/rcan_arch.py:8-135) on the HIP engine.

Module tree and parameter names are the reference's (``body.{g}.residual_group.{b}.rcab.{0,2}``
3x3 convs, ``rcab.3.attention.{1,3}`` squeeze 1x1 convs, ``body.{g}.conv``); each RCAB is one
fused op (ops/blocks.py: conv-ReLU-conv, channel attention, ``*res_scale + x``), each
ResidualGroup's tail conv fuses the group skip, the head/tail fuse the mean shift.
"""
import torch
from torch import nn as nn

from ..ops import blocks as BK
from ..ops import conv as C
from ..utils.registry import ARCH_REGISTRY
from .arch_util import Upsample, make_layer


class ChannelAttention(nn.Module):
    """avg-pool -> 1x1 (C -> C/s) -> ReLU -> 1x1 (C/s -> C) -> sigmoid; x * y (rcan_arch.py:8-24)."""

    def __init__(self, num_feat, squeeze_factor=16):
        super().__init__()
        self.attention = nn.Sequential(
            nn.AdaptiveAvgPool2d(1), nn.Conv2d(num_feat, num_feat // squeeze_factor, 1, padding=0),
            nn.ReLU(inplace=True), nn.Conv2d(num_feat // squeeze_factor, num_feat, 1, padding=0), nn.Sigmoid())


class RCAB(nn.Module):
    """Residual channel attention block (rcan_arch.py:27-46) as one fused HIP op."""

    def __init__(self, num_feat, squeeze_factor=16, res_scale=1):
        super().__init__()
        self.res_scale = res_scale
        self.rcab = nn.Sequential(
            nn.Conv2d(num_feat, num_feat, 3, 1, 1), nn.ReLU(True), nn.Conv2d(num_feat, num_feat, 3, 1, 1),
            ChannelAttention(num_feat, squeeze_factor))

    def forward(self, x):
        att = self.rcab[3].attention
        return BK.rcab(x, self.rcab[0], self.rcab[2], att[1], att[3], self.res_scale)


class ResidualGroup(nn.Module):
    """num_block RCABs + conv + group skip (rcan_arch.py:49-68)."""

    def __init__(self, num_feat, num_block, squeeze_factor=16, res_scale=1):
        super().__init__()
        self.residual_group = make_layer(
            RCAB, num_block, num_feat=num_feat, squeeze_factor=squeeze_factor, res_scale=res_scale)
        self.conv = nn.Conv2d(num_feat, num_feat, 3, 1, 1)

    def forward(self, x):
        return C.conv3x3(self.residual_group(x), self.conv, res=x)


@ARCH_REGISTRY.register()
class RCAN(nn.Module):

    def __init__(self,
                 num_in_ch,
                 num_out_ch,
                 num_feat=64,
                 num_group=10,
                 num_block=16,
                 squeeze_factor=16,
                 upscale=4,
                 res_scale=1,
                 img_range=255.,
                 rgb_mean=(0.4488, 0.4371, 0.4040)):
        super().__init__()
        self.img_range = img_range
        self.mean = torch.Tensor(rgb_mean).view(1, 3, 1, 1)
        self.num_in_ch, self.num_out_ch = num_in_ch, num_out_ch
        self.conv_first = nn.Conv2d(num_in_ch, num_feat, 3, 1, 1)
        self.body = make_layer(
            ResidualGroup,
            num_group,
            num_feat=num_feat,
            num_block=num_block,
            squeeze_factor=squeeze_factor,
            res_scale=res_scale)
        self.conv_after_body = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.upsample = Upsample(upscale, num_feat)
        self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
        self._consts = None

    def forward(self, x):
        if self._consts is None or self._consts[0] != x.device:
            mean = self.mean.reshape(-1).float().to(x.device)
            self._consts = (x.device, mean, C.vec([self.img_range] * self.num_in_ch, x.device),
                            C.inv_range(self.img_range, self.num_out_ch, x.device))
        _, mean, rng, inv = self._consts
        dt = C.feature_dtype()
        h = C.to_nhwc(x, C.pad8(self.num_in_ch), dt, shift=mean, scale=rng)
        x0 = C.conv3x3(h, self.conv_first)
        res = C.conv3x3(self.body(x0), self.conv_after_body, res=x0)
        return C.conv3x3(self.upsample(res), self.conv_last, out_nchw=True, aff_scale=inv, aff_shift=mean)
