"""ORACLE — CPU restatement of the reference SR nets (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the CPU baseline; the product path
(basicsr4rs_amd) never calls it.

Every function restates the reference's forward from its source (file:line cited) as
plain PyTorch-CPU fp32 operations on a state_dict whose keys are the reference's own
parameter names.  The arithmetic of the reference lives in PyTorch (torch==2.1.1,
requirements.txt:1 — nn.Conv2d, nn.PixelShuffle, nn.Linear, nn.LayerNorm, softmax, GELU);
here it runs on the container's torch 2.10 CPU kernels, pinned in tests/test_oracle.py
against independent restatements (oracle/c/conv_ref.c direct convolution, explicit index
loops for the shuffles) and the reference's own shape tests
(tests/test_archs/test_srresnet_arch.py:6-19, tests/test_models/test_sr_model.py:96-125).
The reference itself cannot be executed here: numeric parity against the
reference implementation is therefore "parity unpinned" beyond those checks.
"""
import math

import torch
import torch.nn.functional as F


def conv(x, sd, name, act=None, slope=0.0):
    """nn.Conv2d(C, C', 3, 1, 1) (e.g. basicsr/archs/arch_util.py:78-79)."""
    y = F.conv2d(x, sd[f'{name}.weight'], sd.get(f'{name}.bias'), stride=1, padding=1)
    if act == 'relu':
        y = F.relu(y)
    elif act == 'lrelu':
        y = F.leaky_relu(y, slope)
    return y


def pixel_shuffle(x, r):
    """out[n, c, h*r+i, w*r+j] = x[n, c*r*r + i*r + j, h, w] (nn.PixelShuffle, arch_util.py:136)."""
    b, c, h, w = x.shape
    return x.view(b, c // (r * r), r, r, h, w).permute(0, 1, 4, 2, 5, 3).reshape(b, c // (r * r), h * r, w * r)


def pixel_unshuffle(x, s):
    """basicsr/archs/arch_util.py:217-234."""
    b, c, hh, hw = x.shape
    h, w = hh // s, hw // s
    return x.view(b, c, h, s, w, s).permute(0, 1, 3, 5, 2, 4).reshape(b, c * s * s, h, w)


def upsample(x, sd, prefix, scale):
    """Upsample (arch_util.py:123-142): module indices 0,2,.. are convs, 1,3,.. PixelShuffle."""
    if (scale & (scale - 1)) == 0:
        for i in range(int(math.log(scale, 2))):
            x = pixel_shuffle(conv(x, sd, f'{prefix}.{2 * i}'), 2)
    elif scale == 3:
        x = pixel_shuffle(conv(x, sd, f'{prefix}.0'), 3)
    else:
        raise ValueError(scale)
    return x


def residual_block(x, sd, prefix, res_scale):
    """ResidualBlockNoBN.forward (arch_util.py:85-88)."""
    out = conv(conv(x, sd, f'{prefix}.conv1', act='relu'), sd, f'{prefix}.conv2')
    return x + out * res_scale


def edsr(sd, x, num_block=16, upscale=4, res_scale=1, img_range=255., rgb_mean=(0.4488, 0.4371, 0.4040)):
    """EDSR.forward (basicsr/archs/edsr_arch.py:50-61)."""
    mean = torch.tensor(rgb_mean, dtype=x.dtype).view(1, 3, 1, 1)
    x = (x - mean) * img_range
    x = conv(x, sd, 'conv_first')
    r = x
    for i in range(num_block):
        r = residual_block(r, sd, f'body.{i}', res_scale)
    res = conv(r, sd, 'conv_after_body')
    res = res + x
    x = conv(upsample(res, sd, 'upsample', upscale), sd, 'conv_last')
    return x / img_range + mean


def msrresnet(sd, x, num_block=16, upscale=4):
    """MSRResNet.forward (basicsr/archs/srresnet_arch.py:52-66)."""
    feat = conv(x, sd, 'conv_first', act='lrelu', slope=0.1)
    out = feat
    for i in range(num_block):
        out = residual_block(out, sd, f'body.{i}', 1.0)
    if upscale == 4:
        out = F.leaky_relu(pixel_shuffle(conv(out, sd, 'upconv1'), 2), 0.1)
        out = F.leaky_relu(pixel_shuffle(conv(out, sd, 'upconv2'), 2), 0.1)
    elif upscale in (2, 3):
        out = F.leaky_relu(pixel_shuffle(conv(out, sd, 'upconv1'), upscale), 0.1)
    out = conv(conv(out, sd, 'conv_hr', act='lrelu', slope=0.1), sd, 'conv_last')
    base = F.interpolate(x, scale_factor=upscale, mode='bilinear', align_corners=False)
    return out + base


def channel_attention(x, sd, prefix):
    """ChannelAttention (basicsr/archs/rcan_arch.py:8-24): x * sigmoid(W2 relu(W1 avgpool(x)))."""
    y = x.mean(dim=(2, 3), keepdim=True)
    y = F.conv2d(y, sd[f'{prefix}.attention.1.weight'], sd[f'{prefix}.attention.1.bias'])
    y = F.relu(y)
    y = F.conv2d(y, sd[f'{prefix}.attention.3.weight'], sd[f'{prefix}.attention.3.bias'])
    return x * torch.sigmoid(y)


def rcan(sd, x, num_group=10, num_block=16, upscale=4, res_scale=1, img_range=255.,
         rgb_mean=(0.4488, 0.4371, 0.4040)):
    """RCAN.forward (basicsr/archs/rcan_arch.py:124-135) with RCAB :44-46 and ResidualGroup :66-68."""
    mean = torch.tensor(rgb_mean, dtype=x.dtype).view(1, 3, 1, 1)
    x = (x - mean) * img_range
    x = conv(x, sd, 'conv_first')
    r = x
    for g in range(num_group):
        gin = r
        for b in range(num_block):
            p = f'body.{g}.residual_group.{b}.rcab'
            t = conv(conv(r, sd, f'{p}.0', act='relu'), sd, f'{p}.2')
            t = channel_attention(t, sd, f'{p}.3')
            r = t * res_scale + r
        r = conv(r, sd, f'body.{g}.conv') + gin
    res = conv(r, sd, 'conv_after_body') + x
    x = conv(upsample(res, sd, 'upsample', upscale), sd, 'conv_last')
    return x / img_range + mean


def rdb(x, sd, p):
    """ResidualDenseBlock.forward (basicsr/archs/rrdbnet_arch.py:32-39)."""
    x1 = conv(x, sd, f'{p}.conv1', act='lrelu', slope=0.2)
    x2 = conv(torch.cat((x, x1), 1), sd, f'{p}.conv2', act='lrelu', slope=0.2)
    x3 = conv(torch.cat((x, x1, x2), 1), sd, f'{p}.conv3', act='lrelu', slope=0.2)
    x4 = conv(torch.cat((x, x1, x2, x3), 1), sd, f'{p}.conv4', act='lrelu', slope=0.2)
    x5 = conv(torch.cat((x, x1, x2, x3, x4), 1), sd, f'{p}.conv5')
    return x5 * 0.2 + x


def rrdbnet(sd, x, scale=4, num_block=23):
    """RRDBNet.forward (basicsr/archs/rrdbnet_arch.py:105-119), RRDB :58-63."""
    if scale == 2:
        feat = pixel_unshuffle(x, 2)
    elif scale == 1:
        feat = pixel_unshuffle(x, 4)
    else:
        feat = x
    feat = conv(feat, sd, 'conv_first')
    body = feat
    for i in range(num_block):
        out = body
        for k in (1, 2, 3):
            out = rdb(out, sd, f'body.{i}.rdb{k}')
        body = out * 0.2 + body
    feat = feat + conv(body, sd, 'conv_body')
    feat = conv(F.interpolate(feat, scale_factor=2, mode='nearest'), sd, 'conv_up1', act='lrelu', slope=0.2)
    feat = conv(F.interpolate(feat, scale_factor=2, mode='nearest'), sd, 'conv_up2', act='lrelu', slope=0.2)
    return conv(conv(feat, sd, 'conv_hr', act='lrelu', slope=0.2), sd, 'conv_last')


def l1_loss(pred, target, loss_weight=1.0, reduction='mean'):
    """L1Loss (basicsr/losses/basic_loss.py:27-52) via weighted_loss (loss_util.py)."""
    d = (pred - target).abs()
    if reduction == 'mean':
        return loss_weight * d.mean()
    if reduction == 'sum':
        return loss_weight * d.sum()
    return loss_weight * d


def adam_step(p, g, m, v, step, lr, beta1=0.9, beta2=0.99, eps=1e-8):
    """One torch.optim.Adam step (single-tensor path) on float64 copies, returns new (p, m, v)."""
    m = m + (1 - beta1) * (g - m)
    v = v * beta2 + (1 - beta2) * g * g
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    denom = v.sqrt() / math.sqrt(bc2) + eps
    return p - (lr / bc1) * m / denom, m, v
