"""MSRResNet (basicsr/archs/srresnet_arch.py:8-66) on the HIP engine — the net the reference's
own arch test exercises (tests/test_archs/test_srresnet_arch.py)."""
from torch import nn as nn

from .. import _lib
from ..ops import blocks as BK
from ..ops import conv as C
from ..utils.registry import ARCH_REGISTRY
from .arch_util import ResidualBlockNoBN, default_init_weights, make_layer


@ARCH_REGISTRY.register()
class MSRResNet(nn.Module):

    def __init__(self, num_in_ch=3, num_out_ch=3, num_feat=64, num_block=16, upscale=4):
        super().__init__()
        self.upscale = upscale
        self.num_in_ch, self.num_out_ch = num_in_ch, num_out_ch
        self.conv_first = nn.Conv2d(num_in_ch, num_feat, 3, 1, 1)
        self.body = make_layer(ResidualBlockNoBN, num_block, num_feat=num_feat)
        if self.upscale in [2, 3]:
            self.upconv1 = nn.Conv2d(num_feat, num_feat * self.upscale * self.upscale, 3, 1, 1)
            self.pixel_shuffle = nn.PixelShuffle(self.upscale)
        elif self.upscale == 4:
            self.upconv1 = nn.Conv2d(num_feat, num_feat * 4, 3, 1, 1)
            self.upconv2 = nn.Conv2d(num_feat, num_feat * 4, 3, 1, 1)
            self.pixel_shuffle = nn.PixelShuffle(2)
        self.conv_hr = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
        self.lrelu = nn.LeakyReLU(negative_slope=0.1, inplace=True)
        default_init_weights([self.conv_first, self.upconv1, self.conv_hr, self.conv_last], 0.1)
        if self.upscale == 4:
            default_init_weights(self.upconv2, 0.1)

    def forward(self, x):
        dt = C.feature_dtype()
        lr = dict(act=_lib.ACT_LRELU, slope=0.1)
        h = C.to_nhwc(x, C.pad8(self.num_in_ch), dt)
        out = self.body(C.conv3x3(h, self.conv_first, **lr))
        if self.upscale == 4:
            out = C.conv3x3(out, self.upconv1, out_ps=2, **lr)
            out = C.conv3x3(out, self.upconv2, out_ps=2, **lr)
        else:
            out = C.conv3x3(out, self.upconv1, out_ps=self.upscale, **lr)
        out = C.conv3x3(C.conv3x3(out, self.conv_hr, **lr), self.conv_last, out_nchw=True)
        return BK.bilinear_up_add(out, x, self.upscale)
