"""Shared SR building blocks (mirror of basicsr/archs/arch_util.py).

Parameter containers are the reference's own ``nn.Conv2d`` modules, so state_dict keys,
shapes and initialisation match (``default_init_weights`` = basicsr/archs/arch_util.py:17-45,
``make_layer`` = :48-61).  Forward passes run on NHWC feature maps through the HIP ops in
``basicsr4rs_amd.ops`` (no torch conv / CPU path).
"""
import collections.abc
import math
from itertools import repeat

import torch
from torch import nn as nn
from torch.nn import init as init
from torch.nn.modules.batchnorm import _BatchNorm

from ..ops import conv as C
from ..ops.dcn import ModulatedDeformConvPack, modulated_deform_conv, offset_conv, split_offset_mask
from ..ops.layout import pixel_unshuffle  # noqa: F401  (re-export, arch_util.py:217-234)
from ..utils.logger import get_root_logger


@torch.no_grad()
def default_init_weights(module_list, scale=1, bias_fill=0, **kwargs):
    """kaiming_normal_ * scale for Conv2d/Linear, BN weight 1 (arch_util.py:17-45)."""
    if not isinstance(module_list, list):
        module_list = [module_list]
    for module in module_list:
        for m in module.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                init.kaiming_normal_(m.weight, **kwargs)
                m.weight.data *= scale
                if m.bias is not None:
                    m.bias.data.fill_(bias_fill)
            elif isinstance(m, _BatchNorm):
                init.constant_(m.weight, 1)
                if m.bias is not None:
                    m.bias.data.fill_(bias_fill)


def make_layer(basic_block, num_basic_block, **kwarg):
    """nn.Sequential of identical blocks (arch_util.py:48-61); keys ``{i}.*``."""
    return nn.Sequential(*[basic_block(**kwarg) for _ in range(num_basic_block)])


class ResidualBlockNoBN(nn.Module):
    """x + res_scale * conv2(relu(conv1(x))) (arch_util.py:64-88), one fused HIP op pair."""

    def __init__(self, num_feat=64, res_scale=1, pytorch_init=False):
        super().__init__()
        self.res_scale = res_scale
        self.conv1 = nn.Conv2d(num_feat, num_feat, 3, 1, 1, bias=True)
        self.conv2 = nn.Conv2d(num_feat, num_feat, 3, 1, 1, bias=True)
        self.relu = nn.ReLU(inplace=True)
        if not pytorch_init:
            default_init_weights([self.conv1, self.conv2], 0.1)

    def forward(self, x):
        """x: NHWC feature map [N, H, W, pad8(num_feat)]."""
        return C.res_block(x, self.conv1, self.conv2, self.res_scale)


class Upsample(nn.Sequential):
    """log2(s) x [conv nf->4nf, PixelShuffle(2)] or [conv nf->9nf, PixelShuffle(3)] (arch_util.py:123-142).

    Keeps the reference module list (state_dict ``{0,2}.weight``); the PixelShuffle is fused
    into each conv's store, so one HIP launch per stage.
    """

    def __init__(self, scale, num_feat):
        m = []
        for r in C.upsample_specs(scale):
            m.append(nn.Conv2d(num_feat, r * r * num_feat, 3, 1, 1))
            m.append(nn.PixelShuffle(r))
        super().__init__(*m)

    def forward(self, x):
        mods = list(self)
        for conv, ps in zip(mods[0::2], mods[1::2]):
            x = C.conv3x3(x, conv, out_ps=ps.upscale_factor)
        return x


def _ntuple(n):

    def parse(x):
        if isinstance(x, collections.abc.Iterable):
            return x
        return tuple(repeat(x, n))

    return parse


to_1tuple = _ntuple(1)
to_2tuple = _ntuple(2)
to_3tuple = _ntuple(3)
to_4tuple = _ntuple(4)
to_ntuple = _ntuple


def trunc_normal_(tensor, mean=0., std=1., a=-2., b=2.):
    """Truncated normal init (same distribution as arch_util.py:266-327)."""
    return init.trunc_normal_(tensor, mean=mean, std=std, a=a, b=b)


class DCNv2Pack(ModulatedDeformConvPack):
    """Modulated deformable conv whose offsets and masks come from a second feature map
    (arch_util.py:237-263; EDVR / BasicVSR deformable alignment).

    ``conv_offset(feat)`` -> chunk(3) -> offset = cat(o1, o2), mask = sigmoid(o3); a mean
    absolute offset above 50 is logged as a warning (the reference's divergence check, a host
    read per call as there).  The reference prefers torchvision.ops.deform_conv2d, whose
    sampling (bilinear, zero outside -1 < h < H, offsets interleaved (h, w) per tap) is the
    same arithmetic as modulated_deform_conv: here both are the HIP DCNv2 path."""

    def forward(self, x, feat):
        offset, mask = split_offset_mask(offset_conv(self.conv_offset, feat))
        offset_absmean = torch.mean(torch.abs(offset))
        if offset_absmean > 50:
            get_root_logger().warning(f'Offset abs mean is {offset_absmean}, larger than 50.')
        return modulated_deform_conv(x, offset, mask, self.weight, self.bias, self.stride, self.padding, self.dilation,
                                     self.groups, self.deformable_groups)
