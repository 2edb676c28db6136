"""EDSR (basicsr/archs/edsr_arch.py:8-61) on the HIP engine.

Head: NCHW fp32 -> NHWC with the mean shift ``(x - mean) * img_range`` fused
(edsr_arch.py:51-52).  Body: ResidualBlockNoBN pairs.  ``conv_after_body`` fuses the global
skip ``res += x`` (:55-56).  Upsample: convs with the PixelShuffle fused in the store.
``conv_last`` stores NCHW fp32 with ``x / img_range + mean`` fused (:58-59).
"""
import torch
from torch import nn as nn

from ..ops import conv as C
from ..utils.registry import ARCH_REGISTRY
from .arch_util import ResidualBlockNoBN, Upsample, make_layer


@ARCH_REGISTRY.register()
class EDSR(nn.Module):

    def __init__(self,
                 num_in_ch,
                 num_out_ch,
                 num_feat=64,
                 num_block=16,
                 upscale=4,
                 res_scale=1,
                 img_range=255.,
                 rgb_mean=(0.4488, 0.4371, 0.4040)):
        super().__init__()
        self.img_range = img_range
        self.mean = torch.Tensor(rgb_mean).view(1, 3, 1, 1)
        self.num_in_ch, self.num_out_ch = num_in_ch, num_out_ch
        self.conv_first = nn.Conv2d(num_in_ch, num_feat, 3, 1, 1)
        self.body = make_layer(ResidualBlockNoBN, num_block, num_feat=num_feat, res_scale=res_scale, pytorch_init=True)
        self.conv_after_body = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.upsample = Upsample(upscale, num_feat)
        self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
        self._consts = None

    def _constants(self, device):
        if self._consts is None or self._consts[0] != device:
            mean = self.mean.reshape(-1).float().to(device)
            self._consts = (device, mean, C.vec([self.img_range] * self.num_in_ch, device),
                            C.inv_range(self.img_range, self.num_out_ch, device))
        return self._consts[1:]

    def forward(self, x):
        mean, rng, inv = self._constants(x.device)
        dt = C.feature_dtype()
        h = C.to_nhwc(x, C.pad8(self.num_in_ch), dt, shift=mean, scale=rng)
        x0 = C.conv3x3(h, self.conv_first)
        res = C.conv3x3(self.body(x0), self.conv_after_body, res=x0)
        return C.conv3x3(self.upsample(res), self.conv_last, out_nchw=True, aff_scale=inv, aff_shift=mean)
