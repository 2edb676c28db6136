"""SwinIR (basicsr/archs/swinir_arch.py:14-933) on the HIP engine.

Module tree, parameter/buffer names (``relative_position_index``, ``attn_mask``), constructor
kwargs and initialisation (_init_weights: trunc_normal(0.02) Linear, LN 1/0) follow the
reference so checkpoints load strictly.  Execution: token maps are NHWC feature maps
(channels padded to a multiple of 8, e.g. 180 -> 184); every SwinTransformerBlock is one fused
op (ops/swin.py), RSTB convs fuse the group skip, head/tail fuse the mean shift.
Stochastic depth (drop_path, swinir_arch.py:14-40, :320-321, linear dpr schedule :796) is
applied in training: one device draw per forward gives every block its two per-sample
factors floor(keep + U) / keep, which the fused block applies in its proj / fc2 residual
epilogues (and to the branch gradients in backward).
"""
import math

import torch
import torch.utils.checkpoint
from torch import nn as nn

from .. import _lib
from ..ops import blocks as BK
from ..ops import conv as C
from ..ops import swin as S
from ..utils.registry import ARCH_REGISTRY
from .arch_util import Upsample, to_2tuple, trunc_normal_


def drop_path_factors(drop_prob, rand):
    """floor(keep + U) / keep (swinir_arch.py:21-25, the factor x.div(keep) * floor(keep + U)
    applies to a branch); ``rand`` holds the U[0,1) draws."""
    keep = 1.0 - drop_prob
    return torch.floor(rand + keep) / keep


class _RowScale(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, s):
        ctx.save_for_backward(s)
        ctx.shape = x.shape
        x2 = x.contiguous().view(x.shape[0], -1)
        return S.row_scale(x2, s, 1).view(ctx.shape)

    @staticmethod
    def backward(ctx, dy):
        s, = ctx.saved_tensors
        return S.row_scale(dy.contiguous().view(ctx.shape[0], -1), s, 1).view(ctx.shape), None


class DropPath(nn.Module):
    """Stochastic depth per sample (swinir_arch.py:29-40).  Inside SwinIR the fused blocks apply
    it themselves; this module serves standalone use (HIP row-scale kernel on the device)."""

    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if not self.drop_prob or not self.training:
            return x
        r = torch.rand(x.shape[0], device=x.device, dtype=torch.float32)
        return _RowScale.apply(x, drop_path_factors(self.drop_prob, r))


class Mlp(nn.Module):

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)


def relative_index(ws):
    """(Δh + ws - 1) * (2ws - 1) + (Δw + ws - 1) over row-major tokens (swinir_arch.py:123-133)."""
    ys, xs = torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing='ij')
    ys, xs = ys.flatten(), xs.flatten()
    dy = ys[:, None] - ys[None, :] + ws - 1
    dx = xs[:, None] - xs[None, :] + ws - 1
    return dy * (2 * ws - 1) + dx


def shift_mask(h, w, ws, s):
    """-100 where two tokens of a shifted window come from different regions (swinir_arch.py:262-281)."""
    def regions(L):
        r = torch.zeros(L, dtype=torch.long)
        r[L - ws:L - s] = 1
        r[L - s:] = 2
        return r
    ids = regions(h)[:, None] * 3 + regions(w)[None, :]  # [h, w]
    win = ids.view(h // ws, ws, w // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
    diff = win[:, None, :] - win[:, :, None]
    return torch.where(diff != 0, torch.tensor(-100.0), torch.tensor(0.0))


class WindowAttention(nn.Module):

    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim = dim
        self.window_size = window_size
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim**-0.5
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window_size[0] - 1) * (2 * window_size[1] - 1), num_heads))
        self.register_buffer('relative_position_index', relative_index(window_size[0]))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        trunc_normal_(self.relative_position_bias_table, std=.02)
        self.softmax = nn.Softmax(dim=-1)


class SwinTransformerBlock(nn.Module):

    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0, mlp_ratio=4., qkv_bias=True,
                 qk_scale=None, drop=0., attn_drop=0., drop_path=0., act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        self.mlp_ratio = mlp_ratio
        if min(self.input_resolution) <= self.window_size:
            self.shift_size = 0
            self.window_size = min(self.input_resolution)
        assert 0 <= self.shift_size < self.window_size, 'shift_size must in 0-window_size'
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, window_size=to_2tuple(self.window_size), num_heads=num_heads,
                                    qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0. else nn.Identity()
        self.norm2 = norm_layer(dim)
        mlp_hidden_dim = int(dim * mlp_ratio)
        self.mlp = Mlp(in_features=dim, hidden_features=mlp_hidden_dim, act_layer=act_layer, drop=drop)
        if self.shift_size > 0:
            attn_mask = shift_mask(self.input_resolution[0], self.input_resolution[1], self.window_size,
                                   self.shift_size)
        else:
            attn_mask = None
        self.register_buffer('attn_mask', attn_mask)
        self._geom = S.AttnGeom(dim, num_heads, self.window_size, self.shift_size)
        self._fc1 = S.plain_spec(dim, mlp_hidden_dim)
        self._fc2 = S.plain_spec(mlp_hidden_dim, dim)

    def drop_prob(self):
        return self.drop_path.drop_prob if isinstance(self.drop_path, DropPath) else 0.0

    def forward(self, x):
        return S.swin_block(x, self, self._geom, self._fc1, self._fc2, dp=getattr(self, '_dp', None))


class BasicLayer(nn.Module):

    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4., qkv_bias=True, qk_scale=None,
                 drop=0., attn_drop=0., drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.depth = depth
        self.use_checkpoint = use_checkpoint
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(
                dim=dim, input_resolution=input_resolution, num_heads=num_heads, window_size=window_size,
                shift_size=0 if (i % 2 == 0) else window_size // 2, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
                drop_path=drop_path[i] if isinstance(drop_path, list) else drop_path, norm_layer=norm_layer)
            for i in range(depth)
        ])
        self.downsample = None

    def forward(self, x):
        for blk in self.blocks:
            if self.use_checkpoint and torch.is_grad_enabled():
                # activation checkpointing per block (swinir_arch.py:460-461); the block's DropPath
                # factors of this forward are bound here so the recomputation sees the same ones
                dp = getattr(blk, '_dp', None)
                x = torch.utils.checkpoint.checkpoint(
                    lambda t, b=blk, d=dp: S.swin_block(t, b, b._geom, b._fc1, b._fc2, dp=d), x, use_reentrant=False)
            else:
                x = blk(x)
        return x


class PatchEmbed(nn.Module):
    """flatten(2).transpose(1, 2) (+ LayerNorm): a no-op layout on NHWC tokens (swinir_arch.py:571-610)."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size = to_2tuple(img_size)
        patch_size = to_2tuple(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        return S.token_layernorm(x, self.norm) if self.norm is not None else x


class PatchUnEmbed(nn.Module):

    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size = to_2tuple(img_size)
        patch_size = to_2tuple(patch_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans = in_chans
        self.embed_dim = embed_dim


class RSTB(nn.Module):

    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4., qkv_bias=True, qk_scale=None,
                 drop=0., attn_drop=0., drop_path=0., norm_layer=nn.LayerNorm, downsample=None, use_checkpoint=False,
                 img_size=224, patch_size=4, resi_connection='1conv'):
        super().__init__()
        self.dim = dim
        self.input_resolution = input_resolution
        self.resi_connection = resi_connection
        self.residual_group = BasicLayer(
            dim=dim, input_resolution=input_resolution, depth=depth, num_heads=num_heads, window_size=window_size,
            mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop, attn_drop=attn_drop,
            drop_path=drop_path, norm_layer=norm_layer, downsample=downsample, use_checkpoint=use_checkpoint)
        if resi_connection == '1conv':
            self.conv = nn.Conv2d(dim, dim, 3, 1, 1)
        elif resi_connection == '3conv':
            self.conv = nn.Sequential(
                nn.Conv2d(dim, dim // 4, 3, 1, 1), nn.LeakyReLU(negative_slope=0.2, inplace=True),
                nn.Conv2d(dim // 4, dim // 4, 1, 1, 0), nn.LeakyReLU(negative_slope=0.2, inplace=True),
                nn.Conv2d(dim // 4, dim, 3, 1, 1))
        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=0, embed_dim=dim,
                                      norm_layer=None)
        self.patch_unembed = PatchUnEmbed(img_size=img_size, patch_size=patch_size, in_chans=0, embed_dim=dim,
                                          norm_layer=None)

    def forward(self, x):
        g = self.residual_group(x)
        if self.resi_connection == '1conv':
            return C.conv3x3(g, self.conv, res=x)
        raise NotImplementedError("resi_connection '3conv' is not on the HIP path yet")


class UpsampleOneStep(nn.Sequential):

    def __init__(self, scale, num_feat, num_out_ch, input_resolution=None):
        self.num_feat = num_feat
        self.input_resolution = input_resolution
        super().__init__(nn.Conv2d(num_feat, (scale**2) * num_out_ch, 3, 1, 1), nn.PixelShuffle(scale))


@ARCH_REGISTRY.register()
class SwinIR(nn.Module):

    def __init__(self, img_size=64, patch_size=1, in_chans=3, embed_dim=96, depths=(6, 6, 6, 6), num_heads=(6, 6, 6, 6),
                 window_size=7, mlp_ratio=4., qkv_bias=True, qk_scale=None, drop_rate=0., attn_drop_rate=0.,
                 drop_path_rate=0.1, norm_layer=nn.LayerNorm, ape=False, patch_norm=True, use_checkpoint=False,
                 upscale=2, img_range=1., upsampler='', resi_connection='1conv', **kwargs):
        super().__init__()
        num_in_ch = in_chans
        num_out_ch = in_chans
        num_feat = 64
        self.img_range = img_range
        if in_chans == 3:
            self.mean = torch.Tensor((0.4488, 0.4371, 0.4040)).view(1, 3, 1, 1)
        else:
            self.mean = torch.zeros(1, 1, 1, 1)
        self.upscale = upscale
        self.upsampler = upsampler
        self.window_size = window_size
        self.num_in_ch, self.num_out_ch = num_in_ch, num_out_ch
        self.conv_first = nn.Conv2d(num_in_ch, embed_dim, 3, 1, 1)
        self.num_layers = len(depths)
        self.embed_dim = embed_dim
        self.ape = ape
        self.patch_norm = patch_norm
        self.num_features = embed_dim
        self.mlp_ratio = mlp_ratio
        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=embed_dim,
                                      embed_dim=embed_dim, norm_layer=norm_layer if self.patch_norm else None)
        num_patches = self.patch_embed.num_patches
        patches_resolution = self.patch_embed.patches_resolution
        self.patches_resolution = patches_resolution
        self.patch_unembed = PatchUnEmbed(img_size=img_size, patch_size=patch_size, in_chans=embed_dim,
                                          embed_dim=embed_dim, norm_layer=norm_layer if self.patch_norm else None)
        if self.ape:
            self.absolute_pos_embed = nn.Parameter(torch.zeros(1, num_patches, embed_dim))
            trunc_normal_(self.absolute_pos_embed, std=.02)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.layers = nn.ModuleList()
        for i_layer in range(self.num_layers):
            self.layers.append(
                RSTB(dim=embed_dim, input_resolution=(patches_resolution[0], patches_resolution[1]),
                     depth=depths[i_layer], num_heads=num_heads[i_layer], window_size=window_size,
                     mlp_ratio=self.mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop_rate,
                     attn_drop=attn_drop_rate, drop_path=dpr[sum(depths[:i_layer]):sum(depths[:i_layer + 1])],
                     norm_layer=norm_layer, downsample=None, use_checkpoint=use_checkpoint, img_size=img_size,
                     patch_size=patch_size, resi_connection=resi_connection))
        self.norm = norm_layer(self.num_features)
        if resi_connection == '1conv':
            self.conv_after_body = nn.Conv2d(embed_dim, embed_dim, 3, 1, 1)
        elif resi_connection == '3conv':
            self.conv_after_body = nn.Sequential(
                nn.Conv2d(embed_dim, embed_dim // 4, 3, 1, 1), nn.LeakyReLU(negative_slope=0.2, inplace=True),
                nn.Conv2d(embed_dim // 4, embed_dim // 4, 1, 1, 0), nn.LeakyReLU(negative_slope=0.2, inplace=True),
                nn.Conv2d(embed_dim // 4, embed_dim, 3, 1, 1))
        if self.upsampler == 'pixelshuffle':
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, num_feat, 3, 1, 1), nn.LeakyReLU(inplace=True))
            self.upsample = Upsample(upscale, num_feat)
            self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
        elif self.upsampler == 'pixelshuffledirect':
            self.upsample = UpsampleOneStep(upscale, embed_dim, num_out_ch, (patches_resolution[0],
                                                                            patches_resolution[1]))
        elif self.upsampler == 'nearest+conv':
            assert self.upscale == 4, 'only support x4 now.'
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, num_feat, 3, 1, 1), nn.LeakyReLU(inplace=True))
            self.conv_up1 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_up2 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_hr = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
            self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        else:
            self.conv_last = nn.Conv2d(embed_dim, num_out_ch, 3, 1, 1)
        self.apply(self._init_weights)
        self._consts = None

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def _blocks(self):
        return [blk for layer in self.layers for blk in layer.residual_group.blocks]

    def drop_path_draws(self, n_blocks, batch, device):
        """U[0,1) draws of one training forward: [blocks, 2 (attention / MLP branch), batch]."""
        return torch.rand(n_blocks, 2, batch, device=device, dtype=torch.float32)

    def _set_drop_path(self, batch, device):
        """Give every block with a non-zero rate its (s1, s2) factors for this forward."""
        blocks = self._blocks()
        probs = [blk.drop_prob() for blk in blocks]
        if not (self.training and any(p > 0 for p in probs)):
            for blk in blocks:
                blk._dp = None
            return
        rand = self.drop_path_draws(len(blocks), batch, device)
        cached = getattr(self, '_dp_keep', None)
        if cached is None or cached[0] != (device, tuple(probs)):  # device constant (no H2D copy under capture)
            keep = torch.tensor([1.0 - p for p in probs], dtype=torch.float32).view(-1, 1, 1).to(device)
            self._dp_keep = cached = ((device, tuple(probs)), keep)
        keep = cached[1]
        fac = torch.floor(rand + keep) / keep
        for i, (blk, p) in enumerate(zip(blocks, probs)):
            blk._dp = (fac[i, 0], fac[i, 1]) if p > 0 else None

    def forward_features(self, x):
        self._set_drop_path(x.shape[0], x.device)
        x = self.patch_embed(x)
        if self.ape:
            x = S.add_pos_embed(x, self.absolute_pos_embed, self.embed_dim)
        for layer in self.layers:
            x = layer(x)
        for blk in self._blocks():
            blk._dp = None
        return S.token_layernorm(x, self.norm)

    def forward(self, x):
        dev = x.device
        if self._consts is None or self._consts[0] != dev:
            # the reference broadcasts self.mean ([1, 3 | 1, 1, 1], swinir_arch.py:750-754, 860-861,
            # 918) over the input and output channels: the kernels take one value per channel (a
            # 4-band remote-sensing net has a 1-element zero mean and 4 channels each side)
            mean = self.mean.reshape(-1).float().to(dev)
            mean_in = torch.broadcast_to(mean, (self.num_in_ch, )).contiguous()
            mean_out = torch.broadcast_to(mean, (self.num_out_ch, )).contiguous()
            self._consts = (dev, mean_in, mean_out, C.vec([self.img_range] * self.num_in_ch, dev),
                            C.inv_range(self.img_range, self.num_out_ch, dev))
        _, mean_in, mean, rng, inv = self._consts
        H, W = x.shape[2], x.shape[3]
        if H % self.window_size or W % self.window_size:
            raise ValueError('SwinIR input must be a multiple of window_size (pad it as SwinIRModel.test does)')
        dt = C.feature_dtype()
        h = C.to_nhwc(x, C.pad8(self.num_in_ch), dt, shift=mean_in, scale=rng)
        x0 = C.conv3x3(h, self.conv_first)
        res = C.conv3x3(self.forward_features(x0), self.conv_after_body, res=x0)
        if self.upsampler == 'pixelshuffle':
            u = C.conv3x3(res, self.conv_before_upsample[0], act=_lib.ACT_LRELU, slope=0.01)
            return C.conv3x3(self.upsample(u), self.conv_last, out_nchw=True, aff_scale=inv, aff_shift=mean)
        if self.upsampler == 'nearest+conv':
            lr = dict(act=_lib.ACT_LRELU, slope=0.2)
            u = C.conv3x3(res, self.conv_before_upsample[0], act=_lib.ACT_LRELU, slope=0.01)
            u = C.conv3x3(u, self.conv_up1, in_up=2, **lr)
            u = C.conv3x3(u, self.conv_up2, in_up=2, **lr)
            u = C.conv3x3(u, self.conv_hr, **lr)
            return C.conv3x3(u, self.conv_last, out_nchw=True, aff_scale=inv, aff_shift=mean)
        if self.upsampler == 'pixelshuffledirect':
            s = self.upscale
            conv = self.upsample[0]
            y = C.conv3x3(res, conv)  # [N, H, W, pad8(s*s*out)] in reference channel order c*s*s + i*s + j
            scale = inv.repeat_interleave(s * s)
            shift = mean.repeat_interleave(s * s)
            from ..ops.layout import pixel_shuffle
            return pixel_shuffle(C.to_nchw(y, conv.out_channels, scale=scale, shift=shift), s)
        # denoising / artifact removal head: x + conv_last(res), then un-shift
        out = C.conv3x3(res, self.conv_last, out_nchw=True, aff_scale=inv)
        return BK.bilinear_up_add(out, x, 1)
