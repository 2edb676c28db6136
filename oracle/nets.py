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


# Storage-rounding emulation (diagnostic, tests only): inside ``bf16_storage()`` every tensor the
# HIP bf16 path stores between kernels (a conv's activated output, a fused residual result) is
# rounded to bf16 and widened again, so the oracle shows the error budget of bf16 activations
# alone.  Off by default: the oracle is the exact restatement.
# ``bf16_storage(grads=True)`` also rounds the gradient of every stored tensor (the HIP backward's
# bf16 gradient maps), plus the two rounding points of the attention MFMAs: the probabilities P
# (forward only: the engine packs them to bf16 for the AV product; dP stays fp32) and the score
# gradient dS (backward only); and the MLP's pre-activation gradient dz (the fc2 dgrad's gated
# output) while h = GELU(z) is rounded forward only.
_STORE_DTYPE = [None]
_STORE_GRADS = [False]


class bf16_storage:
    def __init__(self, grads=False):
        self.grads = grads

    def __enter__(self):
        self._prev = (_STORE_DTYPE[0], _STORE_GRADS[0])
        _STORE_DTYPE[0] = torch.bfloat16
        _STORE_GRADS[0] = self.grads
        return self

    def __exit__(self, *exc):
        _STORE_DTYPE[0], _STORE_GRADS[0] = self._prev
        return False


def _round(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _RoundFB(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t):
        return _round(t)

    @staticmethod
    def backward(ctx, g):
        return _round(g)


class _RoundB(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t):
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        return _round(g)


class _RoundF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t):
        return _round(t)

    @staticmethod
    def backward(ctx, g):
        return g


def store(t):
    """A tensor written to HBM between kernels: identity unless bf16_storage() is active."""
    if _STORE_DTYPE[0] is None:
        return t
    if _STORE_GRADS[0] and t.requires_grad:
        return _RoundFB.apply(t)
    return _round(t)


def store_fwd(t):
    """Rounded forward only (a bf16 MFMA operand whose gradient stays fp32)."""
    if _STORE_DTYPE[0] is None:
        return t
    return _RoundF.apply(t) if (_STORE_GRADS[0] and t.requires_grad) else _round(t)


class _GeluAuxRounded(torch.autograd.Function):
    """GELU whose backward multiplies by bf16-rounded GELU'(z): the engine's forward stores GELU'(z)
    in bf16 (the aux map) and the fc2 dgrad's gate reads it."""

    @staticmethod
    def forward(ctx, z):
        ctx.save_for_backward(z)
        return F.gelu(z)

    @staticmethod
    def backward(ctx, g):
        (z, ) = ctx.saved_tensors
        d = 0.5 * (1 + torch.erf(z / math.sqrt(2))) + z * torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi)
        return g * _round(d)


def gelu_stored(z):
    """F.gelu, or under bf16_storage(grads=True) the engine's GELU with its bf16 derivative map."""
    return _GeluAuxRounded.apply(z) if (_STORE_DTYPE[0] is not None and _STORE_GRADS[0] and z.requires_grad) else F.gelu(z)


def store_grad(t):
    """Identity forward, bf16-rounded gradient (a gradient map the backward stores)."""
    return _RoundB.apply(t) if (_STORE_DTYPE[0] is not None and _STORE_GRADS[0] and t.requires_grad) else t


def conv(x, sd, name, act=None, slope=0.0, stored=True):
    """nn.Conv2d(C, C', 3, 1, 1) (e.g. basicsr/archs/arch_util.py:78-79)."""
    y = F.conv2d(x, sd[f'{name}.weight'], sd.get(f'{name}.bias'), stride=1, padding=1)
    if act == 'relu':
        y = F.relu(y)
    elif act == 'lrelu':
        y = F.leaky_relu(y, slope)
    return store(y) if stored else y


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
    x5 = conv(torch.cat((x, x1, x2, x3, x4), 1), sd, f'{p}.conv5', stored=False)
    return store(x5 * 0.2 + x)


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
        body = store(out * 0.2 + body)
    feat = store(feat + conv(body, sd, 'conv_body', stored=False))
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


def _ln(x, sd, p):
    """nn.LayerNorm over the last dim, eps 1e-5."""
    return F.layer_norm(x, (x.shape[-1], ), sd[f'{p}.weight'], sd[f'{p}.bias'], 1e-5)


def _linear(x, sd, p):
    return F.linear(x, sd[f'{p}.weight'], sd.get(f'{p}.bias'))


def window_partition(x, ws):
    """(b, h, w, c) -> (b * nW, ws, ws, c)  (basicsr/archs/swinir_arch.py:63-75)."""
    b, h, w, c = x.shape
    return x.view(b, h // ws, ws, w // ws, ws, c).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws, ws, c)


def window_reverse(windows, ws, h, w):
    """Inverse of window_partition (swinir_arch.py:78-92)."""
    b = windows.shape[0] // ((h // ws) * (w // ws))
    return windows.view(b, h // ws, w // ws, ws, ws, -1).permute(0, 1, 3, 2, 4, 5).reshape(b, h, w, -1)


def rel_index(ws):
    """relative_position_index (swinir_arch.py:123-133)."""
    coords = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing='ij')).flatten(1)
    rel = (coords[:, :, None] - coords[:, None, :]).permute(1, 2, 0)
    return (rel[:, :, 0] + ws - 1) * (2 * ws - 1) + (rel[:, :, 1] + ws - 1)


def swin_mask(h, w, ws, s):
    """calculate_mask (swinir_arch.py:262-281): -100 between tokens of different regions."""
    img = torch.zeros(1, h, w, 1)
    cnt = 0
    for hs in (slice(0, -ws), slice(-ws, -s), slice(-s, None)):
        for wsl in (slice(0, -ws), slice(-ws, -s), slice(-s, None)):
            img[:, hs, wsl, :] = cnt
            cnt += 1
    mw = window_partition(img, ws).view(-1, ws * ws)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)


def window_attention(xw, sd, p, nH, ws, mask):
    """WindowAttention.forward (swinir_arch.py:144-175)."""
    b_, n, c = xw.shape
    hd = c // nH
    qkv = store(_linear(xw, sd, f'{p}.qkv')).reshape(b_, n, 3, nH, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0] * hd**-0.5, qkv[1], qkv[2]
    attn = q @ k.transpose(-2, -1)
    table = sd[f'{p}.relative_position_bias_table']
    bias = table[rel_index(ws).reshape(-1)].view(n, n, -1).permute(2, 0, 1)
    attn = attn + bias.unsqueeze(0)
    if mask is not None:
        nw = mask.shape[0]
        attn = attn.view(b_ // nw, nw, nH, n, n) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, nH, n, n)
    attn = store_fwd(store_grad(attn).softmax(-1))
    out = store((attn @ v).transpose(1, 2).reshape(b_, n, c))
    return _linear(out, sd, f'{p}.proj')


def window_attention_core(qkv, nH, ws, shift, scale, table):
    """The attention core of SwinTransformerBlock + WindowAttention between the qkv Linear
    and the proj Linear (swinir_arch.py:288-314 roll / partition / reverse, :151-172
    scale, q k^T, relative bias, shift mask, softmax, attn @ v), on a token map.
    qkv: [b, h, w, 3*C] with channel order [3][nH][hd] (swinir_arch.py:151); returns the
    head-concatenated output [b, h, w, C] (channel h*hd + d, :172) at the un-shifted pixels."""
    b, h, w, c3 = qkv.shape
    c = c3 // 3
    hd = c // nH
    t = qkv
    if shift > 0:
        t = torch.roll(t, shifts=(-shift, -shift), dims=(1, 2))
    tw = window_partition(t, ws).reshape(-1, ws * ws, 3, nH, hd).permute(2, 0, 3, 1, 4)
    q, k, v = tw[0] * scale, tw[1], tw[2]
    n = ws * ws
    attn = q @ k.transpose(-2, -1)
    attn = attn + table[rel_index(ws).reshape(-1)].view(n, n, -1).permute(2, 0, 1).unsqueeze(0)
    if shift > 0:
        mask = swin_mask(h, w, ws, shift).to(attn.dtype)
        nw = mask.shape[0]
        attn = (attn.view(-1, nw, nH, n, n) + mask.unsqueeze(1).unsqueeze(0)).view(-1, nH, n, n)
    out = (attn.softmax(-1) @ v).transpose(1, 2).reshape(-1, ws, ws, c)
    t = window_reverse(out, ws, h, w)
    if shift > 0:
        t = torch.roll(t, shifts=(shift, shift), dims=(1, 2))
    return t


def drop_path(x, drop_prob, rand):
    """drop_path in training (swinir_arch.py:14-26) with the U[0,1) draws ``rand`` [B] given."""
    if drop_prob == 0.:
        return x
    keep_prob = 1 - drop_prob
    random_tensor = keep_prob + rand.view((x.shape[0], ) + (1, ) * (x.ndim - 1)).to(x.dtype)
    random_tensor.floor_()
    return x.div(keep_prob) * random_tensor


def swin_block(x, sd, p, hw, nH, ws, shift, res=None, dp=None):
    """SwinTransformerBlock.forward (swinir_arch.py:283-323); DropPath = identity (eval) unless
    ``dp`` = (drop_prob, rand [2, B]) gives the training draws of its two branches (:320-321).
    ``res``: the block's constructor input_resolution (img_size / patch_size); the no-shift /
    shrunken-window rule (swinir_arch.py:234-237) is decided on it, not on the runtime size
    ``hw`` (which only sets the shapes and the shift mask, :315-318)."""
    h, w = hw
    b, _, c = x.shape
    res = hw if res is None else res
    if min(res) <= ws:
        shift, ws = 0, min(res)
    sc = x
    t = store(_ln(x, sd, f'{p}.norm1')).view(b, h, w, c)
    if shift > 0:
        t = torch.roll(t, shifts=(-shift, -shift), dims=(1, 2))
    tw = window_partition(t, ws).view(-1, ws * ws, c)
    aw = window_attention(tw, sd, f'{p}.attn', nH, ws, swin_mask(h, w, ws, shift) if shift > 0 else None)
    t = window_reverse(aw.view(-1, ws, ws, c), ws, h, w)
    if shift > 0:
        t = torch.roll(t, shifts=(shift, shift), dims=(1, 2))
    t = t.reshape(b, h * w, c)
    m_fn = lambda v: _linear(store_fwd(gelu_stored(store_grad(_linear(store(_ln(v, sd, f'{p}.norm2')), sd, f'{p}.mlp.fc1')))),  # noqa: E731
                             sd, f'{p}.mlp.fc2')
    if dp is not None:
        x = store(sc + drop_path(t, dp[0], dp[1][0]))
        return store(x + drop_path(m_fn(x), dp[0], dp[1][1]))
    x = store(sc + t)
    return store(x + m_fn(x))


def swinir(sd, x, cfg, dp_rand=None):
    """SwinIR.forward (swinir_arch.py:868-922), 1conv residual (ape optional); eval mode, or training
    stochastic depth when ``dp_rand`` [blocks, 2, B] holds the U[0,1) draws (rates: the linear
    schedule torch.linspace(0, drop_path_rate, sum(depths)), swinir_arch.py:796)."""
    in_ch = cfg.get('in_chans', 3)
    img_range = cfg.get('img_range', 1.)
    ws = cfg.get('window_size', 7)
    depths, heads = cfg.get('depths', (6, 6, 6, 6)), cfg.get('num_heads', (6, 6, 6, 6))
    ups, s = cfg.get('upsampler', ''), cfg.get('upscale', 2)
    mean = torch.tensor((0.4488, 0.4371, 0.4040)).view(1, 3, 1, 1) if in_ch == 3 else torch.zeros(1, 1, 1, 1)
    x = (x - mean) * img_range
    b, _, h, w = x.shape
    img = cfg.get('img_size', 64)
    img = (img, img) if isinstance(img, int) else tuple(img)
    res = (img[0] // cfg.get('patch_size', 1), img[1] // cfg.get('patch_size', 1))

    dpr = [v.item() for v in torch.linspace(0, cfg.get('drop_path_rate', 0.1), sum(depths))]

    def features(f):
        t = f.flatten(2).transpose(1, 2)
        if cfg.get('patch_norm', True):
            t = store(_ln(t, sd, 'patch_embed.norm'))
        if cfg.get('ape', False):  # swinir_arch.py:879-880
            t = t + sd['absolute_pos_embed']
        k = 0
        for i, d in enumerate(depths):
            g = t
            for j in range(d):
                dp = (dpr[k], dp_rand[k]) if dp_rand is not None else None
                g = swin_block(g, sd, f'layers.{i}.residual_group.blocks.{j}', (h, w), heads[i], ws,
                               0 if j % 2 == 0 else ws // 2, res=res, dp=dp)
                k += 1
            g = g.transpose(1, 2).reshape(b, -1, h, w)
            t = store(conv(g, sd, f'layers.{i}.conv', stored=False).flatten(2).transpose(1, 2) + t)
        t = store(_ln(t, sd, 'norm'))
        return t.transpose(1, 2).reshape(b, -1, h, w)

    if ups == 'pixelshuffle':
        x = conv(x, sd, 'conv_first')
        x = conv(features(x), sd, 'conv_after_body') + x
        x = F.leaky_relu(conv(x, sd, 'conv_before_upsample.0'), 0.01)
        x = conv(upsample(x, sd, 'upsample', s), sd, 'conv_last')
    elif ups == 'pixelshuffledirect':
        x = conv(x, sd, 'conv_first')
        x = conv(features(x), sd, 'conv_after_body') + x
        x = pixel_shuffle(conv(x, sd, 'upsample.0'), s)
    elif ups == 'nearest+conv':
        x = conv(x, sd, 'conv_first')
        x = conv(features(x), sd, 'conv_after_body') + x
        x = F.leaky_relu(conv(x, sd, 'conv_before_upsample.0'), 0.01)
        x = conv(F.interpolate(x, scale_factor=2, mode='nearest'), sd, 'conv_up1', act='lrelu', slope=0.2)
        x = conv(F.interpolate(x, scale_factor=2, mode='nearest'), sd, 'conv_up2', act='lrelu', slope=0.2)
        x = conv(conv(x, sd, 'conv_hr', act='lrelu', slope=0.2), sd, 'conv_last')
    else:
        xf = conv(x, sd, 'conv_first')
        res = conv(features(xf), sd, 'conv_after_body') + xf
        x = x + conv(res, sd, 'conv_last')
    return x / img_range + mean
