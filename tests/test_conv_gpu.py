"""GPU parity of the HIP 3x3 conv path against the CPU oracle (torch fp32 restatement).

Tolerances: fp32 mode runs exact-f32 MFMA (v_mfma_f32_16x16x4_f32) and differs from the
CPU only by summation order -> |err| <= 1e-4 * max(1, |ref|max).  bf16 mode rounds inputs
and weights to bf16 (8 significant bits) and accumulates in fp32 -> compared against the
oracle evaluated on the same bf16-rounded operands, |err| <= 2e-2 * |ref|max.
"""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from basicsr4rs_amd import _lib
from basicsr4rs_amd.ops import conv as C
from basicsr4rs_amd.ops.layout import pixel_shuffle, pixel_unshuffle
from oracle import nets as O

pytestmark = pytest.mark.gpu


def nhwc_to_nchw_t(y, c):
    return y[..., :c].permute(0, 3, 1, 2).float()


def rel_err(a, b):
    return (a - b).abs().max().item() / max(1.0, b.abs().max().item())


def bf(t):
    return t.to(torch.bfloat16).float()


CASES = [
    # (N, H, W, cin, cout, kwargs)
    (2, 16, 16, 64, 64, {}),
    (1, 12, 20, 3, 64, {}),
    (2, 8, 8, 24, 40, {'act': _lib.ACT_RELU}),
    (1, 16, 16, 64, 48, {'act': _lib.ACT_LRELU, 'slope': 0.2}),
    (2, 8, 8, 64, 256, {'out_ps': 2}),
    (1, 8, 8, 32, 288, {'out_ps': 3}),
    (2, 16, 16, 64, 3, {'out_nchw': True}),
    (1, 64, 64, 256, 256, {}),
]


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', CASES)
def test_conv3x3_fwd_bwd(cuda, case, dtype):
    N, H, W, cin, cout, kw = case
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, 3, 1, 1)
    x = torch.randn(N, cin, H, W)
    w, b = conv.weight.detach(), conv.bias.detach()
    if dtype == torch.bfloat16:
        xr, wr = bf(x), bf(w)
    else:
        xr, wr = x.clone(), w
    xr.requires_grad_(True)
    wr = wr.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    ref = F.conv2d(xr, wr, br, padding=1)
    if kw.get('act') == _lib.ACT_RELU:
        ref = F.relu(ref)
    elif kw.get('act') == _lib.ACT_LRELU:
        ref = F.leaky_relu(ref, kw['slope'])
    if kw.get('out_ps'):
        ref = O.pixel_shuffle(ref, kw['out_ps'])
    g = torch.randn_like(ref)
    (ref * g).sum().backward()

    gconv = copy.deepcopy(conv).to(cuda)
    xg = x.to(cuda).requires_grad_(True)
    h = C.to_nhwc(xg, C.pad8(cin), dtype)
    y = C.conv3x3(h, gconv, **kw)
    if kw.get('out_nchw'):
        yn = y
    else:
        yn = nhwc_to_nchw_t(y, ref.shape[1])
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert yn.shape == ref.shape
    assert rel_err(yn.cpu(), ref.detach()) < tol
    (yn * g.to(cuda)).sum().backward()
    assert rel_err(gconv.weight.grad.cpu(), wr.grad) < tol * 2
    assert rel_err(gconv.bias.grad.cpu(), br.grad) < tol * 2
    assert rel_err(xg.grad.cpu(), xr.grad) < tol * 2


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_residual_block(cuda, dtype):
    from basicsr4rs_amd.archs.arch_util import ResidualBlockNoBN
    torch.manual_seed(1)
    blk = ResidualBlockNoBN(64, res_scale=0.1)
    x = torch.randn(2, 64, 16, 16)
    sd = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    if dtype == torch.bfloat16:
        sd = {k: (bf(v) if k.endswith('weight') else v) for k, v in sd.items()}
        xr = bf(x)
    else:
        xr = x
    sd = {k: v.requires_grad_(True) for k, v in sd.items()}
    xr = xr.clone().requires_grad_(True)
    sd2 = {f'blk.{k}': v for k, v in sd.items()}
    ref = O.residual_block(xr, sd2, 'blk', 0.1)
    g = torch.randn_like(ref)
    (ref * g).sum().backward()
    gb = copy.deepcopy(blk).to(cuda)
    xg = x.to(cuda).requires_grad_(True)
    h = C.to_nhwc(xg, 64, dtype)
    y = nhwc_to_nchw_t(gb(h), 64)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert rel_err(y.cpu(), ref.detach()) < tol
    (y * g.to(cuda)).sum().backward()
    assert rel_err(xg.grad.cpu(), xr.grad) < tol * 2
    for n, p in gb.named_parameters():
        assert rel_err(p.grad.cpu(), sd[n].grad) < tol * 4, n


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('r', [2, 3])
def test_pixel_shuffle_bit_exact(cuda, dtype, r):
    x = torch.randn(2, 4 * r * r, 5, 7, dtype=dtype)
    y = pixel_shuffle(x.to(cuda), r).cpu()
    assert torch.equal(y, O.pixel_shuffle(x, r))
    assert torch.equal(y, nn.PixelShuffle(r)(x))
    z = pixel_unshuffle(y.to(cuda), r).cpu()
    assert torch.equal(z, x)
    assert torch.equal(z, O.pixel_unshuffle(y, r))


def test_edsr_m_parity_fp32(cuda):
    from basicsr4rs_amd.archs import build_network
    torch.manual_seed(42)
    net = build_network(dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=4, upscale=4))
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in net.state_dict().items()}
    x = torch.rand(1, 3, 64, 64, generator=torch.Generator().manual_seed(0))
    gt = torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(1))
    ref = O.edsr(sd, x, num_block=4, upscale=4)
    O.l1_loss(ref, gt).backward()
    gnet = copy.deepcopy(net).to(cuda)
    out = gnet(x.to(cuda))
    err = (out.cpu() - ref.detach()).abs().max().item()
    assert err < 1e-3, err
    mse = ((out.cpu() - ref.detach())**2).mean().item()
    psnr = 10 * torch.log10(torch.tensor(1.0 / max(mse, 1e-20))).item()
    assert psnr > 60, psnr
    (out - gt.to(cuda)).abs().mean().backward()
    for n, p in gnet.named_parameters():
        assert rel_err(p.grad.cpu(), sd[n].grad) < 1e-3, n


@pytest.mark.parametrize('shape', [(2, 64, 64, 256, 256, 0, 3), (1, 20, 36, 256, 512, 0, 3), (3, 17, 9, 256, 768, 0, 3),
                                   (1, 16, 16, 1024, 256, 2, 3), (2, 8, 24, 256, 1024, 2, 3),
                                   (1, 12, 20, 264, 256, 0, 3), (2, 16, 16, 64, 256, 0, 1), (1, 9, 15, 184, 544, 0, 1),
                                   (2, 8, 16, 576, 184, 0, 1), (1, 9, 15, 368, 184, 0, 1), (1, 5, 13, 368, 544, 0, 1)])
def test_big_tile_kernel_bitwise_equals_small(cuda, shape):
    """The phase-interleaved 256x256 kernel (variant 24: never the halo form), the 128x128
    register-staged kernel (1) and the two-barrier 256x256 kernel (2) sum K in the same order,
    so their bf16 outputs must be bitwise identical (partial M/N tiles, K-steps crossing taps,
    a single K-step, 1x1 taps, in_ps gather).  1x1 shapes with K > 192 and Cout >= 128
    (SwinIR fc2 / qkv and fc1 dgrads) take the 256x256 kernels with a partial N tile."""
    N, H, W, cin, cout, in_ps, ks = shape
    torch.manual_seed(3)
    dt = torch.bfloat16
    lib = _lib.load()
    if in_ps:
        x = torch.randn(N, H * in_ps, W * in_ps, cin // (in_ps * in_ps), device=cuda).to(dt)
    else:
        x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    taps = 9 if ks == 3 else 1
    wf = (torch.randn(cout, taps * cin, device=cuda) * 0.05).to(dt)
    bg = torch.randn(cout, device=cuda)
    res = torch.randn(N, H, W, cout, device=cuda).to(dt)
    outs = []
    try:
        for variant in (24, 1, 2):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            y = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
            C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout, res=res, alpha=0.5, in_ps=in_ps, ldx=x.shape[-1],
                           ksize=ks)
            outs.append(y)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])


@pytest.mark.parametrize('shape', [(2, 16, 16, 256, 256, 0), (1, 20, 12, 512, 256, 0), (2, 9, 14, 256, 768, 0),
                                   (1, 8, 12, 256, 1024, 2), (1, 3, 64, 256, 256, 0), (2, 3, 128, 256, 1024, 2),
                                   (1, 5, 64, 384, 256, 0)])
@pytest.mark.parametrize('variant', [0, 1, 2])
def test_wgrad_bf16_vs_fp64(cuda, shape, variant):
    """Weight/bias gradient (256x256 LDS-DMA kernels: phase-interleaved = variant 0 where
    W % 64 == 0, two-barrier = variant 2; small kernel = variant 1)
    against an fp64 CPU reference on the same bf16-rounded operands; |err| <= 1e-2*|ref|max."""
    N, H, W, cin, cout, ps = shape
    torch.manual_seed(5)
    dt = torch.bfloat16
    lib = _lib.load()
    x = torch.randn(N, H, W, cin).to(dt)
    if ps:
        dy = torch.randn(N, H * ps, W * ps, cout // (ps * ps)).to(dt)
        dy_gemm = O.pixel_unshuffle(dy.permute(0, 3, 1, 2).double(), ps)  # [N, cout, H, W], channel c*r*r+s
    else:
        dy = torch.randn(N, H, W, cout).to(dt)
        dy_gemm = dy.permute(0, 3, 1, 2).double()
    xd = x.permute(0, 3, 1, 2).double()
    w = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
    F.conv2d(xd, w, b, padding=1).mul(dy_gemm).sum().backward()
    _lib.check(lib.sr_conv3x3_set_variant(variant))
    try:
        dw, db = C.conv_wgrad_raw(dy.to(cuda), x.to(cuda), N, H, W, cin, cin, cout, cout, scale=1.0, out_ps=ps)
        torch.cuda.synchronize()
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    assert rel_err(dw.cpu().double(), w.grad) < 1e-2 * max(1.0, w.grad.abs().max().item()) / max(1.0, w.grad.abs().max().item())
    assert (dw.cpu().double() - w.grad).abs().max().item() <= 1e-3 * w.grad.abs().max().item() + 1e-3
    assert (db.cpu().double() - b.grad).abs().max().item() <= 1e-3 * b.grad.abs().max().item() + 1e-3


@pytest.mark.parametrize('shape', [(2, 4, 64, 256, 256, 0), (1, 3, 128, 256, 1024, 2), (1, 7, 64, 256, 512, 0)])
def test_wgrad_pp_bitwise_equals_big(cuda, shape):
    """The phase-interleaved wgrad kernel sums each pixel K-step in the same order as the
    two-barrier 256x256 kernel (same splits, same MFMA chain): slabs, dW and db bitwise equal."""
    N, H, W, cin, cout, ps = shape
    torch.manual_seed(11)
    dt = torch.bfloat16
    lib = _lib.load()
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    dy = torch.randn(N, H * max(ps, 1), W * max(ps, 1), cout // max(ps * ps, 1), device=cuda).to(dt)
    outs = []
    try:
        for variant in (78, 2):  # 78: the pp kernel where the kernel-row wgrad would run
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            outs.append(C.conv_wgrad_raw(dy, x, N, H, W, cin, cin, cout, cout, scale=1.0, out_ps=ps))
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize('shape', [(1, 3, 64, 256, 256), (4, 8, 64, 256, 256), (2, 64, 64, 256, 256),
                                   (8, 64, 64, 256, 256), (1, 6, 64, 128, 256), (2, 5, 128, 128, 512),
                                   (1, 7, 192, 384, 256), (3, 1, 64, 256, 512), (1, 4, 64, 256, 1024, 2),
                                   (2, 3, 128, 256, 1024, 2), (1, 2, 64, 128, 2304, 3)])
def test_wgrad_row3_vs_fp64(cuda, shape):
    """Kernel-row weight gradient (conv3x3_wgrad_row3_kernel: three taps of a 256 x 128 tile per
    block from one x halo row per 64-pixel step; bias-role blocks) against an fp64 reference on the
    same bf16 operands, and against the pp kernel (variant 78) within fp32 summation-order noise:
    one-step splits, splits crossing images, image rows of one pixel row (H 1), W 64 / 128 / 192,
    Cin 128 / 384, two co tiles, several bias-group sizes; pixel-shuffled dy (r 2 / 3: the EDSR upsample
    convs' GEMM columns, one shuffle slot per 256-co tile)."""
    N, H, W, cin, cout = shape[:5]
    ps = shape[5] if len(shape) > 5 else 0
    torch.manual_seed(21)
    dt = torch.bfloat16
    lib = _lib.load()
    x = torch.randn(N, H, W, cin).to(dt)
    if ps:
        dy = torch.randn(N, H * ps, W * ps, cout // (ps * ps)).to(dt)
        dy_gemm = O.pixel_unshuffle(dy.permute(0, 3, 1, 2).double(), ps)
    else:
        dy = torch.randn(N, H, W, cout).to(dt)
        dy_gemm = dy.permute(0, 3, 1, 2).double()
    w = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.permute(0, 3, 1, 2).double(), w, b, padding=1).mul(dy_gemm).sum().backward()
    d = _lib.WgradDesc()
    d.dtype, d.N, d.H, d.W = _lib.dtype_code(dt), N, H, W
    d.Cin, d.Cin_real, d.ldx, d.Cout, d.Cout_real, d.ldy, d.ksize = cin, cin, cin, cout, cout, dy.shape[-1], 3
    d.out_ps = ps
    assert lib.sr_conv3x3_wgrad_kernel_name(d) == b'conv3x3_wgrad_row3_kernel'
    outs = []
    try:
        for variant, bg in ((0, -1), (0, 1), (0, 5), (78, -1)):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            with _lib.knob('SR_WG_ROW3', bg):
                outs.append(C.conv_wgrad_raw(dy.to(cuda), x.to(cuda), N, H, W, cin, cin, cout, cout, scale=1.0,
                                             out_ps=ps))
                torch.cuda.synchronize()
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    scale = w.grad.abs().max().item()
    for dw, db in outs[:3]:
        assert (dw.cpu().double() - w.grad).abs().max().item() <= 2e-5 * scale + 1e-4
        assert (db.cpu().double() - b.grad).abs().max().item() <= 2e-5 * b.grad.abs().max().item() + 1e-4
    for dw, db in outs[1:]:  # bias-group sizes change the split plan (and the fp32 summation order) only
        assert (outs[0][0] - dw).abs().max().item() <= 2e-5 * scale + 1e-4


@pytest.mark.parametrize('shape', [(2, 64, 64, 180, 180), (1, 8, 128, 180, 180), (2, 16, 64, 136, 180)])
def test_conv_kpad_pph_vs_halo_and_fp64(cuda, shape, monkeypatch):
    """SwinIR-M's 180 -> 180 3x3 conv (stored as 184 channels) with a residual: with K-padded weight
    images (ops.conv._kpad: GEMM K 192, the x rows keeping their 184-channel stride) the forward runs
    on the halo-row 256x256 kernel with a partial output tile (the dgrad stays on the halo kernel);
    against the 64-channel halo kernel (SR_CONV_KPAD=0) and a float64 conv of the same bf16 operands:
    y, dx, dW, db."""
    from basicsr4rs_amd.utils import ktrace
    N, H, W, cin, cout = shape
    torch.manual_seed(7)
    conv = nn.Conv2d(cin, cout, 3, 1, 1)
    x = torch.zeros(N, H, W, C.pad8(cin))
    x[..., :cin] = torch.randn(N, H, W, cin)
    x = x.to(torch.bfloat16)
    res = torch.zeros(N, H, W, C.pad8(cout))
    res[..., :cout] = torch.randn(N, H, W, cout)
    res = res.to(torch.bfloat16)
    gy = torch.zeros(N, H, W, C.pad8(cout))
    gy[..., :cout] = torch.randn(N, H, W, cout)
    gy = gy.to(torch.bfloat16)
    outs = {}
    for kp in ('1', '0'):
        monkeypatch.setenv('SR_CONV_KPAD', kp)
        c = copy.deepcopy(conv).to(cuda)
        xx = x.to(cuda).requires_grad_()
        ktrace.start()
        try:
            y = C.conv3x3(xx, c, res=res.to(cuda))
            y.backward(gy.to(cuda))
            torch.cuda.synchronize()
        finally:
            ran = set(ktrace.stop())
        assert ('conv3x3_fwd_pph_kernel' in ran) == (kp == '1'), ran
        outs[kp] = (y.float().cpu()[..., :cout], xx.grad.float().cpu()[..., :cin], c.weight.grad.cpu(),
                    c.bias.grad.cpu())
    xd = x[..., :cin].permute(0, 3, 1, 2).double().requires_grad_()
    wd = conv.weight.detach().to(torch.bfloat16).double().requires_grad_()
    bd = conv.bias.detach().double().requires_grad_()
    yd = F.conv2d(xd, wd, bd, padding=1) + res[..., :cout].permute(0, 3, 1, 2).double()
    yd.backward(gy[..., :cout].permute(0, 3, 1, 2).double())
    ref = (yd.detach().permute(0, 2, 3, 1), xd.grad.permute(0, 2, 3, 1), wd.grad, bd.grad)
    for kp in ('1', '0'):
        for got, want in zip(outs[kp], ref):
            scale = want.abs().max().item()
            assert (got.double() - want).abs().max().item() <= 1e-2 * scale, kp
    for a, b in zip(outs['1'], outs['0']):  # the two kernels: within bf16 rounding of each other
        assert (a - b).abs().max().item() <= 1e-2 * b.abs().max().item()


@pytest.mark.parametrize('shape', [(2, 64, 64, 184, 576), (1, 64, 64, 192, 184), (3, 8, 64, 184, 360),
                                   (1, 8, 64, 360, 184), (1, 5, 13, 64, 64), (1, 3, 7, 200, 72),
                                   (4, 32, 32, 384, 384), (1, 1, 1, 64, 64)])
def test_linear_wgrad_vs_fp64(cuda, shape):
    """1x1 weight / bias gradient on linear_wgrad_kernel (192x192 tiles over token K-ranges; SwinIR
    qkv / proj / fc1 / fc2 shapes, partial channel tiles, ragged token counts down to one) against
    fp64 on the same bf16 operands and against the 256x256 pp kernel (variant 63)."""
    N, H, W, cin, cout = shape
    torch.manual_seed(14)
    dt = torch.bfloat16
    lib = _lib.load()
    x = torch.randn(N, H, W, cin).to(dt)
    dy = torch.randn(N, H, W, cout).to(dt)
    d = _lib.WgradDesc()
    d.dtype, d.N, d.H, d.W = _lib.dtype_code(dt), N, H, W
    d.Cin, d.Cin_real, d.ldx, d.Cout, d.Cout_real, d.ldy, d.out_ps, d.ksize = cin, cin, cin, cout, cout, cout, 0, 1
    assert lib.sr_conv3x3_wgrad_kernel_name(d) == b'linear_wgrad_kernel'
    outs = []
    try:
        for variant in (0, 63):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            outs.append(C.conv_wgrad_raw(dy.to(cuda), x.to(cuda), N, H, W, cin, cin, cout, cout, scale=1.0, ksize=1))
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    xd, dyd = x.double().reshape(-1, cin), dy.double().reshape(-1, cout)
    ref_w, ref_b = dyd.t() @ xd, dyd.sum(0)
    torch.cuda.synchronize()
    dw, db = outs[0]
    dw = dw.cpu().double().reshape(cout, cin)
    assert (dw - ref_w).abs().max().item() <= 1e-3 * ref_w.abs().max().item() + 1e-3
    assert (db.cpu().double() - ref_b).abs().max().item() <= 1e-3 * ref_b.abs().max().item() + 1e-3
    assert (dw - outs[1][0].cpu().double().reshape(cout, cin)).abs().max().item() <= 1e-3 * ref_w.abs().max().item() + 1e-3


@pytest.mark.parametrize('shape', [(2, 6, 64, 256, 256), (1, 4, 128, 128, 192), (32, 8, 64, 256, 256),
                                   (3, 3, 64, 8, 256), (1, 5, 64, 96, 128), (2, 64, 64, 256, 256),
                                   (2, 5, 64, 184, 184), (1, 3, 128, 184, 72), (2, 6, 64, 64, 256, 2),
                                   (1, 4, 128, 64, 256, 2), (3, 2, 64, 32, 256, 2), (1, 3, 64, 64, 576, 3)])
def test_wgrad_ring_wide_vs_fp64(cuda, shape):
    """Row-streaming wgrad over 64-channel output tiles (Cout above 64, the last tile partial: the
    EDSR-L body shape, SwinIR's 184-channel convs; variant 62 forces it) against fp64 on the same bf16 operands and against the default
    kernel; image top / bottom rows, multi-image splits, Cin below one 64-channel chunk, and (round 3)
    pixel-shuffled dy (the RCAN / SwinIR upsample convs 64 -> 256, r 2: each co tile inside one slot)."""
    N, H, W, cin, cout = shape[:5]
    ps = shape[5] if len(shape) > 5 else 0
    torch.manual_seed(13)
    dt = torch.bfloat16
    lib = _lib.load()
    x = torch.randn(N, H, W, cin).to(dt)
    if ps:
        dy = torch.randn(N, H * ps, W * ps, cout // (ps * ps)).to(dt)
        dy_gemm = O.pixel_unshuffle(dy.permute(0, 3, 1, 2).double(), ps)
    else:
        dy = torch.randn(N, H, W, cout).to(dt)
        dy_gemm = dy.permute(0, 3, 1, 2).double()
    d = _lib.WgradDesc()
    d.dtype, d.N, d.H, d.W = _lib.dtype_code(dt), N, H, W
    d.Cin, d.Cin_real, d.ldx, d.Cout, d.Cout_real, d.ldy, d.out_ps, d.ksize = cin, cin, cin, cout, cout, dy.shape[-1], ps, 3
    outs = []
    try:
        _lib.check(lib.sr_conv3x3_set_variant(62))
        assert lib.sr_conv3x3_wgrad_kernel_name(d) == b'conv3x3_wgrad_ring_kernel'
        for variant in (62, 0, 67):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            outs.append(C.conv_wgrad_raw(dy.to(cuda), x.to(cuda), N, H, W, cin, cin, cout, cout, scale=1.0, out_ps=ps))
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    w = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.permute(0, 3, 1, 2).double(), w, b, padding=1).mul(dy_gemm).sum().backward()
    torch.cuda.synchronize()
    dw, db = outs[0]
    assert (dw.cpu().double() - w.grad).abs().max().item() <= 1e-3 * w.grad.abs().max().item() + 1e-3
    assert (db.cpu().double() - b.grad).abs().max().item() <= 1e-3 * b.grad.abs().max().item() + 1e-3
    for other in outs[1:]:  # the automatic choice, and variant 67 (no shuffled-dy ring)
        assert (dw - other[0]).abs().max().item() <= 1e-3 * w.grad.abs().max().item() + 1e-3
        assert (db - other[1]).abs().max().item() <= 1e-3 * b.grad.abs().max().item() + 1e-3


@pytest.mark.parametrize('shape', [(2, 3, 64, 64, 64, 1), (1, 2, 128, 192, 32, 1), (1, 5, 64, 160, 48, 1),
                                   (1, 3, 64, 64, 16, 1), (1, 2, 128, 64, 64, 2), (3, 1, 64, 96, 8, 1),
                                   (3, 20, 64, 64, 32, 1), (2, 10, 256, 64, 64, 1), (4, 12, 128, 96, 32, 2),
                                   (16, 16, 64, 64, 64, 1), (6, 22, 64, 192, 32, 1), (4, 32, 128, 64, 64, 2)])
def test_wgrad_halo_vs_fp64(cuda, shape):
    """All-taps halo wgrad (Cout <= 64, W % 64 == 0), row-streaming form: channel slices of
    wider buffers (ldx, xcoff, ldy, ycoff as in RRDB dense blocks), nearest-x2 input gather
    (in_up = 2), splits that cross image boundaries (rows per split not dividing H), several
    64-px column segments per row, ragged last split, against an fp64 CPU reference on the same
    bf16 operands; a repeat call is bitwise equal (the split slab reduce is in a fixed order)."""
    N, H, W, cin, cout, up = shape
    torch.manual_seed(9)
    dt = torch.bfloat16
    lib = _lib.load()
    xw = torch.randn(N, H // up, W // up, cin + 24).to(dt)  # x = channels [8, 8 + cin) of a wider map
    dyw = torch.randn(N, H, W, cout + 16).to(dt)            # dy = channels [16, 16 + cout)
    x = xw[..., 8:8 + cin]
    dy = dyw[..., 16:16 + cout]
    xd = x.permute(0, 3, 1, 2).double()
    if up > 1:
        xd = F.interpolate(xd, scale_factor=up, mode='nearest')
    w = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
    F.conv2d(xd, w, b, padding=1).mul(dy.permute(0, 3, 1, 2).double()).sum().backward()
    d = _lib.WgradDesc()
    d.dtype, d.N, d.H, d.W, d.ksize, d.in_up = _lib.dtype_code(dt), N, H, W, 3, up
    d.Cin = d.Cin_real = cin
    d.Cout = d.Cout_real = cout
    d.ldx, d.xcoff, d.ldy, d.ycoff = cin + 24, 8, cout + 16, 16
    assert lib.sr_conv3x3_wgrad_kernel_name(d) == b'conv3x3_wgrad_ring_kernel'
    runs = [C.conv_wgrad_raw(dyw.to(cuda), xw.to(cuda), N, H, W, cin, cin, cout, cout, scale=1.0, ldx=cin + 24,
                             xcoff=8, ldy=cout + 16, ycoff=16, in_up=up) for _ in range(2)]
    torch.cuda.synchronize()
    dw, db = runs[0]
    assert torch.equal(dw, runs[1][0]) and torch.equal(db, runs[1][1])
    tol = 1e-3 * w.grad.abs().max().item() + 1e-3
    assert (dw.cpu().double() - w.grad).abs().max().item() <= tol
    assert (db.cpu().double() - b.grad).abs().max().item() <= 1e-3 * b.grad.abs().max().item() + 1e-3


@pytest.mark.parametrize('shape', [(2, 8, 64, 64, 64), (1, 4, 128, 192, 32), (1, 4, 64, 96, 48), (2, 4, 64, 160, 8),
                                   (1, 6, 128, 64, 64), (1, 4, 128, 32, 96), (1, 4, 128, 32, 192),
                                   (2, 8, 64, 64, 160), (1, 4, 64, 184, 184)])
@pytest.mark.parametrize('epi', ['plain', 'relu_res'])
def test_fwd_halo_vs_fp64(cuda, shape, epi):
    """Narrow-conv halo forward (Cout <= 64, W 64/128): channel-slice input (ldx > Cin, xcoff),
    output written into a slice of a wider buffer (RRDB dense layout), bias + LeakyReLU or
    residual epilogues, ragged Cin chunks, against fp64 on the same bf16 operands; and
    bitwise equal to the 128-row register-staged kernel when Cin == 64 (same K order)."""
    N, H, W, cin, cout = shape
    torch.manual_seed(4)
    dt = torch.bfloat16
    lib = _lib.load()
    conv = nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    spec = C.ConvSpec(cin, cout)
    wf, wd, bg = C.prepared(conv.weight, conv.bias, spec, dt)
    xw = torch.randn(N, H, W, cin + 16, device=cuda).to(dt)
    x = xw[..., 8:8 + cin]
    res = torch.randn(N, H, W, cout, device=cuda).to(dt)
    ldy = cout + 24
    kw = dict(ldx=cin + 16, xcoff=8, ldy=ldy, ycoff=16)
    if epi == 'relu_res':
        kw.update(act=_lib.ACT_LRELU, slope=0.2, res=res, alpha=0.2, beta=1.0)
    outs = []
    try:
        for variant in (0, 1):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            y = torch.zeros(N, H, W, ldy, device=cuda, dtype=dt)
            C.conv_fwd_raw(xw, wf, bg, y, N, H, W, cin, cout, cout, **kw)
            outs.append(y)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    xd = x.permute(0, 3, 1, 2).double().cpu()
    ref = F.conv2d(xd, bf(conv.weight.detach().cpu()).double(), conv.bias.detach().cpu().double(), padding=1)
    if epi == 'relu_res':
        ref = 0.2 * F.leaky_relu(ref, 0.2) + res.permute(0, 3, 1, 2).double().cpu()
    got = outs[0][..., 16:16 + cout].permute(0, 3, 1, 2).double().cpu()
    assert (got - ref).abs().max().item() <= 2e-2 * max(1.0, ref.abs().max().item())
    assert outs[0][..., :16].abs().max().item() == 0 and outs[0][..., 16 + cout:].abs().max().item() == 0
    if cin == 64:
        assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize('case', [(torch.bfloat16, 2, 8, 64, 64, 64), (torch.bfloat16, 2, 16, 16, 64, 64),
                                  (torch.float32, 2, 16, 16, 64, 64), (torch.bfloat16, 1, 16, 16, 256, 256),
                                  (torch.bfloat16, 2, 16, 16, 64, 16), (torch.bfloat16, 1, 8, 128, 64, 32)])
def test_fwd_colsum_matches_output(cuda, case):
    """Fused per-image channel sums (RCAN avg-pool input) of every conv kernel family: summed
    over their partial rows they equal the channel sums of y as stored."""
    dt, N, H, W, cin, cout = case
    torch.manual_seed(5)
    lib = _lib.load()
    conv = nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    spec = C.ConvSpec(cin, cout)
    wf, _, bg = C.prepared(conv.weight, conv.bias, spec, dt)
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    y = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
    d = C._desc(dt, N, H, W, cin, cin, cout, cout, cout)
    P = lib.sr_conv3x3_fwd_colsum_parts(d)
    assert P > 0
    y2, parts = C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout, act=_lib.ACT_RELU, colsum=True)
    assert parts.shape == (N, P, cout)
    ref = y.double().sum((1, 2))
    got = parts.double().sum(1)
    tol = 1e-5 * y.double().abs().sum((1, 2)).max().item() + 1e-6
    assert (got - ref).abs().max().item() <= tol


def test_refresh_prepared_matches_fresh_prep(cuda):
    """The one-launch rebuild of every cached weight image after an optimizer step (conv,
    pixel-shuffled conv, mapped linear) equals per-weight preparation, and re-keys the cache."""
    from basicsr4rs_amd.ops import swin as SW
    torch.manual_seed(6)
    dt = torch.bfloat16
    lib = _lib.load()
    c1, c2 = nn.Conv2d(64, 64, 3, 1, 1).to(cuda), nn.Conv2d(64, 256, 3, 1, 1).to(cuda)
    lin = nn.Linear(180, 540).to(cuda)
    s1, s2 = C.ConvSpec(64, 64), C.ConvSpec(64, 256, out_ps=2)
    ls = SW.qkv_spec(180, 6, 32)
    C.prepared(c1.weight, c1.bias, s1, dt)
    C.prepared(c2.weight, c2.bias, s2, dt)
    SW.prepared_linear(lin.weight, lin.bias, ls, dt)
    with torch.no_grad():  # an optimizer writing behind autograd's back (no version bump)
        for m in (c1, c2, lin):
            m.weight.data.mul_(-1.5).add_(0.25)
            m.bias.data.add_(1.0)
    C.bump_param_epoch()
    C.refresh_prepared()
    got = [C.prepared(c1.weight, c1.bias, s1, dt), C.prepared(c2.weight, c2.bias, s2, dt),
           SW.prepared_linear(lin.weight, lin.bias, ls, dt)]
    rm, cm, _, _ = ls.maps(cuda)
    for (w, b, shape, maps), imgs in zip([(c1.weight, c1.bias, (64, 64, 64, 64, 0, 3), (None, None)),
                                          (c2.weight, c2.bias, (256, 64, 256, 64, 2, 3), (None, None)),
                                          (lin.weight, lin.bias, (540, 180, ls.cout_p, ls.cin_p, 0, 1), (rm, cm))],
                                         got):
        cr, ci, cp, cip, ops, ks = shape
        taps = 9 if ks == 3 else 1
        wf = torch.empty(cp, taps * cip, device=cuda, dtype=dt)
        wd = torch.empty(cip, taps * cp, device=cuda, dtype=dt)
        bg = torch.empty(cp, device=cuda)
        _lib.check(lib.sr_conv_prep_mapped(_lib.dtype_code(dt), ks, _lib.ptr(w.detach()), _lib.ptr(b.detach()), cr, ci,
                                           cp, cip, ops, _lib.ptr(maps[0]), _lib.ptr(maps[1]), _lib.ptr(wf),
                                           _lib.ptr(wd), _lib.ptr(bg), _lib.stream()))
        assert torch.equal(imgs[0], wf) and torch.equal(imgs[1], wd) and torch.equal(imgs[2], bg)


@pytest.mark.parametrize('shape', [(2, 64, 64, 256, 256), (1, 8, 64, 256, 1024), (2, 4, 64, 512, 256),
                                   (1, 12, 64, 64, 384), (3, 4, 64, 128, 256), (1, 6, 128, 256, 256),
                                   (2, 2, 128, 128, 512), (1, 4, 128, 64, 256)])
def test_fwd_pph_vs_fp64(cuda, shape):
    """Halo form of the 256x256 kernel (W 64 / 128 whole-row tiles, chunk-major K): against fp64 on
    the same bf16 operands, with a channel-slice input, residual + LeakyReLU epilogue and the
    fused channel sums; close to the tap-major pp kernel (only the K summation order differs)."""
    N, H, W, cin, cout = shape
    torch.manual_seed(9)
    dt = torch.bfloat16
    lib = _lib.load()
    xw = torch.randn(N, H, W, cin + 16, device=cuda).to(dt)
    x = xw[..., 8:8 + cin]
    wt = torch.randn(cout, cin, 3, 3, device=cuda) * 0.05
    bias = torch.randn(cout, device=cuda)
    spec = C.ConvSpec(cin, cout)
    wf, _, bg = C.prepared(torch.nn.Parameter(wt), torch.nn.Parameter(bias), spec, dt)
    res = torch.randn(N, H, W, cout, device=cuda).to(dt)
    d = C._desc(dt, N, H, W, cin, cin + 16, cout, cout, cout)
    assert lib.sr_conv3x3_fwd_kernel_name(d) == b'conv3x3_fwd_pph_kernel'
    outs = []
    try:
        for variant in (0, 24):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            y = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
            _, parts = C.conv_fwd_raw(xw, wf, bg, y, N, H, W, cin, cout, cout, ldx=cin + 16, xcoff=8,
                                      act=_lib.ACT_LRELU, slope=0.2, res=res, beta=1.0, colsum=True)
            outs.append((y, parts))
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    xd = x.permute(0, 3, 1, 2).double().cpu()
    ref = F.conv2d(xd, bf(wt.cpu()).double(), bias.cpu().double(), padding=1)
    ref = F.leaky_relu(ref, 0.2) + res.permute(0, 3, 1, 2).double().cpu()
    y0, p0 = outs[0]
    got = y0.permute(0, 3, 1, 2).double().cpu()
    assert (got - ref).abs().max().item() <= 2e-2 * max(1.0, ref.abs().max().item())
    assert (y0.float() - outs[1][0].float()).abs().max().item() <= 2e-2 * max(1.0, ref.abs().max().item())
    cs = y0.double().sum((1, 2))
    assert (p0.double().sum(1) - cs).abs().max().item() <= 1e-5 * y0.double().abs().sum((1, 2)).max().item()


@pytest.mark.parametrize('shape', [(2, 4, 64, 184, 576), (1, 4, 64, 192, 184), (1, 2, 128, 368, 184),
                                   (2, 2, 64, 184, 368), (1, 3, 64, 128, 136)])
def test_wgrad_1x1_partial_tiles_vs_fp64(cuda, shape):
    """Linear-layer weight gradients on the 256x256 kernel (variant 63: linear_wgrad_kernel off) with
    partial co / ci tiles (SwinIR qkv / proj / fc1 / fc2 shapes): dW = dy^T x and db = sum dy against fp64, and equal to
    the 128x128 kernel (variant 28) within bf16-operand rounding."""
    N, H, W, cin, cout = shape
    torch.manual_seed(7)
    dt = torch.bfloat16
    lib = _lib.load()
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    dy = torch.randn(N, H, W, cout, device=cuda).to(dt)
    d = _lib.WgradDesc()
    d.dtype, d.N, d.H, d.W, d.Cin, d.Cin_real, d.ldx, d.Cout, d.Cout_real, d.ldy, d.ksize = (
        _lib.SR_BF16, N, H, W, cin, cin, cin, cout, cout, cout, 1)
    ref_w = dy.reshape(-1, cout).double().cpu().t() @ x.reshape(-1, cin).double().cpu()
    ref_b = dy.reshape(-1, cout).double().cpu().sum(0)
    outs = []
    try:
        _lib.check(lib.sr_conv3x3_set_variant(63))  # linear_wgrad_kernel off: the pp kernel
        assert lib.sr_conv3x3_wgrad_kernel_name(d) == b'conv3x3_wgrad_pp_kernel'
        for variant in (63, 28):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            dw, db = C.conv_wgrad_raw(dy, x, N, H, W, cin, cin, cout, cout, ksize=1)
            outs.append((dw.reshape(cout, cin).cpu().double(), db.cpu().double()))
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    for dw, db in outs:
        assert (dw - ref_w).abs().max().item() <= 1e-3 * ref_w.abs().max().item() + 1e-3
        assert (db - ref_b).abs().max().item() <= 1e-3 * ref_b.abs().max().item() + 1e-3


@pytest.mark.parametrize('shape', [(2, 3, 256, 256, 3), (1, 2, 256, 64, 3), (1, 2, 256, 96, 16), (2, 40, 512, 128, 3),
                                   (1, 33, 256, 256, 16), (3, 35, 256, 64, 8), (32, 256, 256, 256, 3),
                                   (32, 256, 256, 64, 3)])
def test_fwd_halo_w256_nchw_tail(cuda, shape):
    """HR-resolution tail conv (conv_last: Cout <= 16, W >= 256, fp32 NCHW store with the mean
    shift / range affine): the row-streaming tail kernel (Cin 64 / 128 / 256; bands of 32 rows,
    ragged last band) or the one-row halo tiles (other Cin, W 256), against fp64 and the 256x16
    kernel (variant 29)."""
    N, H, W, cin, cout = shape
    torch.manual_seed(11)
    dt = torch.bfloat16
    lib = _lib.load()
    conv = nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    scale = torch.rand(cout, device=cuda) + 0.5
    shift = torch.randn(cout, device=cuda)
    spec = C.ConvSpec(cin, cout, out_nchw=True)
    wf, _, bg = C.prepared(conv.weight, conv.bias, spec, dt)
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    d = C._desc(dt, N, H, W, cin, cin, spec.cout_p, cout, 0, out_nchw=1)
    want = b'conv3x3_fwd_tail_kernel' if cin in (64, 128, 256) else b'conv3x3_fwd_halo_kernel'
    assert lib.sr_conv3x3_fwd_kernel_name(d) == want
    outs = []
    try:
        for variant in (0, 29):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            y = torch.empty(N, cout, H, W, device=cuda)
            C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, spec.cout_p, cout, out_nchw=True, aff_scale=scale,
                           aff_shift=shift)
            outs.append(y)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    # full-size cases (the EDSR_Lx4 / RCAN / SwinIR conv_last at B 32: 8 blocks per CU, each block's
    # ring prologue racing the previous block's LDS contents): fp64 on the first and last image
    im = [0, N - 1] if N > 4 else list(range(N))
    ref = F.conv2d(x[im].permute(0, 3, 1, 2).double().cpu(), bf(conv.weight.detach().cpu()).double(),
                   conv.bias.detach().cpu().double(), padding=1)
    ref = ref * scale.cpu().double().view(1, -1, 1, 1) + shift.cpu().double().view(1, -1, 1, 1)
    tol = 1e-3 * max(1.0, ref.abs().max().item())
    assert torch.isfinite(outs[0]).all()
    assert (outs[0][im].cpu().double() - ref).abs().max().item() <= tol
    assert (outs[0] - outs[1]).abs().max().item() <= tol


@pytest.mark.parametrize('shape', [(4, 64, 64, 3, 64), (2, 32, 48, 3, 256), (1, 16, 16, 1, 64)])
@pytest.mark.parametrize('variant', [0, 33])
def test_wgrad_rgb_head_reduce_vs_fp64(cuda, shape, variant):
    """Weight/bias gradient of the RGB head conv (Cin_real 3 or 1, padded to 8 channels): the
    block-per-channel slab reduce (variant 0) and the one-thread-per-weight reduce (33) against
    fp64 on the same bf16 operands."""
    N, H, W, cin_real, cout = shape
    torch.manual_seed(11)
    dt = torch.bfloat16
    lib = _lib.load()
    x = torch.zeros(N, H, W, 8)
    x[..., :cin_real] = torch.randn(N, H, W, cin_real)
    x = x.to(dt)
    dy = torch.randn(N, H, W, cout).to(dt)
    xd = x[..., :cin_real].permute(0, 3, 1, 2).double()
    w = torch.zeros(cout, cin_real, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
    F.conv2d(xd, w, b, padding=1).mul(dy.permute(0, 3, 1, 2).double()).sum().backward()
    _lib.check(lib.sr_conv3x3_set_variant(variant))
    try:
        dw, db = C.conv_wgrad_raw(dy.to(cuda), x.to(cuda), N, H, W, 8, cin_real, cout, cout, scale=1.0)
        torch.cuda.synchronize()
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    dw = dw.cpu().double().reshape(w.shape)
    assert (dw - w.grad).abs().max().item() <= 1e-3 * w.grad.abs().max().item() + 1e-3
    assert (db.cpu().double() - b.grad).abs().max().item() <= 1e-3 * b.grad.abs().max().item() + 1e-3


def _same_or_ulp(a, b, exact):
    """Bitwise equal, or (a different fp32 summation order before the bf16 store) within one bf16
    rounding step of the larger magnitude plus 1e-3 of the tensor's range for cancelled values."""
    if exact:
        assert torch.equal(a, b)
        return
    a, b = a.float(), b.float()
    tol = torch.maximum(a.abs(), b.abs()) * 2.0 ** -7 + 1e-3 * a.abs().max().item()
    assert bool(((a - b).abs() <= tol).all()), (a - b).abs().max().item()


@pytest.mark.parametrize('shape', [(16, 64, 64, 64, 64), (5, 13, 64, 64, 64), (1, 1, 64, 64, 64), (3, 2, 64, 32, 32),
                                   (2, 24, 128, 64, 32), (2, 9, 128, 32, 64), (4, 7, 64, 32, 64), (2, 9, 128, 32, 96),
                                   (3, 5, 128, 64, 192), (2, 6, 64, 32, 160)])
@pytest.mark.parametrize('epi', ['relu', 'gate_alpha_res', 'gelu_gate_aux', 'res2_rowscale', 'colsum', 'slices',
                                 'rrdb_dgrad'])
@pytest.mark.parametrize('grid', [36, 35])
def test_fwd_band_bitwise_equals_halo(cuda, shape, epi, grid):
    """Row-streaming narrow conv (conv3x3_fwd_band_kernel: persistent bands of image rows, 4-slot
    LDS row ring, epilogue operands staged by LDS-DMA) against the tile kernel it replaces
    (variant 34) -- same K order, so bitwise equal (Cout <= 32: see _same_or_ulp) -- on every
    epilogue the nets use, with bands
    of one row (variant 36: 256 blocks, one row each on small shapes) and long bands crossing image
    boundaries (variant 35: 64 blocks); colsum partial rows sum to the stored output's channel
    sums."""
    N, H, W, cin, cout = shape
    if cout > 64 and epi == 'colsum':
        pytest.skip('fused channel sums are not sliced (RCAN convs are 64 wide)')
    torch.manual_seed(6)
    dt = torch.bfloat16
    lib = _lib.load()
    conv = nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    wf, _, bg = C.prepared(conv.weight, conv.bias, C.ConvSpec(cin, cout), dt)
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    gate = torch.randn(N, H, W, cout, device=cuda).to(dt)
    res = torch.randn(N, H, W, cout, device=cuda).to(dt)
    res2 = torch.randn(N, H, W, cout, device=cuda).to(dt)
    kw, ldy, ycoff, xin = {}, cout, 0, x
    if epi == 'relu':
        kw = dict(act=_lib.ACT_RELU)
    elif epi == 'gate_alpha_res':
        kw = dict(gate=gate, gate_slope=0.2, alpha=0.3, res=res, beta=0.7)
    elif epi == 'gelu_gate_aux':
        kw = dict(gate=gate, gate_mode=1, aux=torch.empty(N, H, W, cout, device=cuda, dtype=dt))
    elif epi == 'res2_rowscale':
        kw = dict(res=res, res2=res2, beta2=-0.5, row_scale=torch.rand(N, device=cuda) * 2)
    elif epi == 'rrdb_dgrad':  # RRDB dense-block dgrad: post-residual LeakyReLU gate on the last 32 columns
        kw = dict(alpha=0.2, res=res, beta=1.0, rcols=min(64, cout), gate=gate, gate_slope=0.2, gate_mode=2,
                  gcol0=cout - 32, gcol1=cout)
    elif epi == 'slices':
        xin = torch.randn(N, H, W, cin + 32, device=cuda).to(dt)
        ldy, ycoff = cout + 24, 16
        kw = dict(ldx=cin + 32, xcoff=16, act=_lib.ACT_LRELU, slope=0.2)
    outs = []
    try:
        for variant in (grid, 34):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            y = torch.zeros(N, H, W, ldy, device=cuda, dtype=dt)
            if variant == grid:
                name = lib.sr_conv3x3_fwd_kernel_name(C._desc(dt, N, H, W, cin, cin, cout, cout, cout)).decode()
                assert name == 'conv3x3_fwd_band_kernel', name
            if epi == 'colsum':
                has = lib.sr_conv3x3_fwd_colsum_parts(C._desc(dt, N, H, W, cin, cin, cout, cout, cout)) > 0
                if has:
                    y, parts = C.conv_fwd_raw(xin, wf, bg, y, N, H, W, cin, cout, cout, colsum=True)
                else:  # the tile kernel has no fused sums at this H * W
                    assert variant == 34
                    y, parts = C.conv_fwd_raw(xin, wf, bg, y, N, H, W, cin, cout, cout), None
                outs.append((y, parts))
            else:
                kk = dict(kw)
                if 'aux' in kk:
                    kk['aux'] = torch.zeros_like(kk['aux'])
                C.conv_fwd_raw(xin, wf, bg, y, N, H, W, cin, cout, cout, ycoff=ycoff, **kk)
                outs.append((y, kk.get('aux')))
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    (y0, e0), (y1, e1) = outs
    # the halo kernel's Cout <= 32 form sums K in 32-channel chunks (three blocks per CU), the band
    # kernel in 64-channel ones: bitwise equal up to Cin 32, within one bf16 rounding step beyond
    _same_or_ulp(y0, y1, exact=cout > 32 or cin <= 32)
    if epi == 'gelu_gate_aux':
        _same_or_ulp(e0, e1, exact=cout > 32 or cin <= 32)
    if epi == 'colsum':
        ref = y0.double().sum((1, 2))
        for parts in (e0, e1):
            if parts is None:
                continue
            got = parts.double().sum(1)
            assert (got - ref).abs().max().item() <= 1e-5 * y0.double().abs().sum((1, 2)).max().item() + 1e-6
    if epi == 'slices':
        assert y0[..., :16].abs().max().item() == 0 and y0[..., 16 + cout:].abs().max().item() == 0


@pytest.mark.parametrize('cin', [64, 96, 128, 160, 192])
@pytest.mark.parametrize('act', [0, 1])
def test_fwd_halo_cout32_vs_fp64(cuda, cin, act):
    """The halo kernel's Cout-32 form (32-channel K chunks in 64-B halo rows, three blocks per CU;
    the RRDB dense convs 2-5 -> 32) against float64 on the same bf16 operands: relative L2 within
    bf16 output rounding (<= 4e-3) and every element within two bf16 steps plus 1e-3 of the range --
    a dropped chunk or a wrong chunk swizzle moves whole channels by O(1)."""
    N, H, W, cout = 3, 20, 128, 32
    torch.manual_seed(12)
    dt = torch.bfloat16
    lib = _lib.load()
    conv = nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    wf, _, bg = C.prepared(conv.weight, conv.bias, C.ConvSpec(cin, cout), dt)
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    kw = dict(act=_lib.ACT_LRELU, slope=0.2) if act else {}
    try:
        _lib.check(lib.sr_conv3x3_set_variant(34))
        name = lib.sr_conv3x3_fwd_kernel_name(C._desc(dt, N, H, W, cin, cin, cout, cout, cout)).decode()
        assert name == 'conv3x3_fwd_halo_kernel', name
        y = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
        C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout, **kw)
        torch.cuda.synchronize()
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    ref = F.conv2d(x.permute(0, 3, 1, 2).double().cpu(), bf(conv.weight.detach().cpu()).double(),
                   conv.bias.detach().cpu().double(), padding=1)
    if act:
        ref = F.leaky_relu(ref, 0.2)
    got = y.permute(0, 3, 1, 2).double().cpu()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel <= 4e-3, rel
    tol = ref.abs() * 2.0 ** -7 + 1e-3 * ref.abs().max().item()
    assert bool(((got - ref).abs() <= tol).all()), (got - ref).abs().max().item()


@pytest.mark.parametrize('shape', [(2, 6, 256, 1, 64, 64), (1, 5, 512, 1, 64, 64), (3, 7, 384, 1, 64, 64),
                                   (2, 4, 256, 2, 64, 64), (1, 6, 128, 2, 64, 64), (2, 8, 512, 2, 64, 64),
                                   (2, 5, 512, 1, 8, 64), (1, 6, 256, 1, 32, 64), (2, 5, 256, 1, 8, 256),
                                   (1, 3, 384, 1, 16, 192), (1, 4, 256, 1, 8, 128)])
@pytest.mark.parametrize('epi', ['plain', 'lrelu', 'gate'])
@pytest.mark.parametrize('grid', [0, 35])
def test_fwd_band_strips_vs_fp64(cuda, shape, epi, grid):
    """64-channel-output convs on images wider than 128 px, and W 128 with the nearest x2 upsample
    folded in: the band kernel over 128-px column strips (the RRDBNet HR convs conv_up1 / conv_up2 /
    conv_hr, their dgrads and conv_last's 8-channel dgrads; from 8 channels into 128 / 256 in one launch
    (EDSR's conv_last dgrad), into 192 as 64-channel output slices) -- each strip's border columns loaded from
    its neighbours, zeros at the image edges; strip rows crossing strips and images inside a band with
    variant 35 (64 blocks) -- against float64 on the same bf16 operands (relative L2 <= 4e-3 and every
    element within two bf16 steps plus 1e-3 of the range: a wrong border column or strip origin moves
    a whole pixel column by O(1)) and against the generic tile kernel it replaces (variant 76) within
    one bf16 rounding step."""
    N, H, W, up, cin, cout = shape
    if cin < 64 and epi == 'lrelu':
        pytest.skip('narrow-input strips: plain and gated (dgrad) epilogues only')
    torch.manual_seed(31)
    dt = torch.bfloat16
    lib = _lib.load()
    conv = nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    wf, _, bg = C.prepared(conv.weight, conv.bias, C.ConvSpec(cin, cout), dt)
    x = torch.randn(N, H // up, W // up, cin, device=cuda).to(dt)
    gate = torch.randn(N, H, W, cout, device=cuda).to(dt)
    kw = {'plain': {}, 'lrelu': dict(act=_lib.ACT_LRELU, slope=0.2),
          'gate': dict(gate=gate, gate_slope=0.2, alpha=0.5)}[epi]
    if up > 1:
        kw['in_up'] = up
    outs = []
    try:
        for variant in (grid, 76):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            d = C._desc(dt, N, H, W, cin, cin, cout, cout, cout, in_up=up if up > 1 else 0)
            name = lib.sr_conv3x3_fwd_kernel_name(d).decode()
            assert (name == 'conv3x3_fwd_band_kernel') == (variant != 76), (variant, name)
            # (the query is pointer-free: a gated call into 128 / 256 channels runs 64-channel slices)
            assert lib.sr_conv3x3_fwd_launches(d) == (cout // 64 if cout == 192 and variant != 76 else 1)
            y = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
            C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout, **kw)
            outs.append(y)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    xd = x.permute(0, 3, 1, 2).double().cpu()
    if up > 1:
        xd = F.interpolate(xd, scale_factor=up, mode='nearest')
    ref = F.conv2d(xd, bf(conv.weight.detach().cpu()).double(), conv.bias.detach().cpu().double(), padding=1)
    if epi == 'lrelu':
        ref = F.leaky_relu(ref, 0.2)
    elif epi == 'gate':
        ref = ref * 0.5 * torch.where(gate.permute(0, 3, 1, 2).double().cpu() > 0, 1.0, 0.2)
    got = outs[0].permute(0, 3, 1, 2).double().cpu()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel <= 4e-3, rel
    tol = ref.abs() * 2.0 ** -7 + 1e-3 * ref.abs().max().item()
    assert bool(((got - ref).abs() <= tol).all()), (got - ref).abs().max().item()
    _same_or_ulp(outs[0], outs[1], exact=False)


@pytest.mark.parametrize('shape', [(2, 4, 64, 1024, 256, 2), (1, 2, 128, 1024, 256, 2), (1, 4, 64, 2304, 256, 3)])
def test_fwd_pph_pixel_shuffled_input(cuda, shape):
    """The halo-row kernel reading a pixel-shuffled input (in_ps: the upsample convs' dgrads read
    the HR gradient as an LR map of r*r*C' channels, LR channel sl*C' + c = HR pixel (y r + sl / r,
    x r + sl % r) channel c): against fp64 on the same bf16 operands and against the per-tap pp
    kernel (variant 50)."""
    N, H, W, cin, cout, r = shape
    torch.manual_seed(21)
    dt = torch.bfloat16
    lib = _lib.load()
    cp = cin // (r * r)
    xh = torch.randn(N, H * r, W * r, cp, device=cuda).to(dt)
    wt = torch.randn(cout, cin, 3, 3, device=cuda) * 0.03
    spec = C.ConvSpec(cin, cout)
    wf, _, bg = C.prepared(torch.nn.Parameter(wt), None, spec, dt)
    d = C._desc(dt, N, H, W, cin, cp, cout, cout, cout, in_ps=r)
    assert lib.sr_conv3x3_fwd_kernel_name(d) == b'conv3x3_fwd_pph_kernel'
    outs = []
    try:
        for variant in (0, 50):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            y = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
            C.conv_fwd_raw(xh, wf, None, y, N, H, W, cin, cout, cout, in_ps=r, ldx=cp)
            outs.append(y)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    xl = xh.view(N, H, r, W, r, cp).permute(0, 2, 4, 5, 1, 3).reshape(N, r * r * cp, H, W)
    ref = F.conv2d(xl.double().cpu(), bf(wt.cpu()).double(), padding=1)
    got = outs[0].permute(0, 3, 1, 2).double().cpu()
    tol = 2e-2 * max(1.0, ref.abs().max().item())
    assert (got - ref).abs().max().item() <= tol
    assert (outs[0].float() - outs[1].float()).abs().max().item() <= tol


@pytest.mark.parametrize('shape', [(2, 4, 64, 256, 64, 2), (1, 6, 128, 256, 64, 2), (2, 4, 64, 576, 64, 3),
                                   (1, 2, 128, 256, 32, 2)])
def test_fwd_halo_pixel_shuffled_input(cuda, shape):
    """The narrow halo kernel reading a pixel-shuffled input (the RCAN / SwinIR upsample convs' dgrads
    into 64 channels: a 64-channel chunk is one shuffle slot, its halo pixels r HR pixels apart): against
    fp64 on the same bf16 operands and against the tile kernel (variant 68)."""
    N, H, W, cin, cout, r = shape
    torch.manual_seed(22)
    dt = torch.bfloat16
    lib = _lib.load()
    cp = cin // (r * r)
    xh = torch.randn(N, H * r, W * r, cp, device=cuda).to(dt)
    wt = torch.randn(cout, cin, 3, 3, device=cuda) * 0.03
    res = torch.randn(N, H, W, cout, device=cuda).to(dt)
    spec = C.ConvSpec(cin, cout)
    wf, _, bg = C.prepared(torch.nn.Parameter(wt), None, spec, dt)
    d = C._desc(dt, N, H, W, cin, cp, cout, cout, cout, in_ps=r)
    assert lib.sr_conv3x3_fwd_kernel_name(d) == b'conv3x3_fwd_halo_kernel'
    outs = []
    try:
        for variant in (0, 68):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            y = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
            C.conv_fwd_raw(xh, wf, None, y, N, H, W, cin, cout, cout, in_ps=r, ldx=cp, res=res, beta=1.0)
            outs.append(y)
        assert lib.sr_conv3x3_fwd_kernel_name(d) != b'conv3x3_fwd_halo_kernel'
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    xl = xh.view(N, H, r, W, r, cp).permute(0, 2, 4, 5, 1, 3).reshape(N, r * r * cp, H, W)
    ref = F.conv2d(xl.double().cpu(), bf(wt.cpu()).double(), padding=1) + res.permute(0, 3, 1, 2).double().cpu()
    got = outs[0].permute(0, 3, 1, 2).double().cpu()
    tol = 2e-2 * max(1.0, ref.abs().max().item())
    assert (got - ref).abs().max().item() <= tol
    assert (outs[0].float() - outs[1].float()).abs().max().item() <= tol


@pytest.mark.parametrize('shape', [(2, 8, 256, 256, 256, 0), (1, 4, 512, 64, 256, 0), (1, 8, 192, 128, 256, 0),
                                   (1, 4, 256, 256, 1024, 2), (3, 12, 320, 64, 320, 0)])
@pytest.mark.parametrize('epi', ['plain', 'relu_res'])
def test_fwd_pph_strips(cuda, shape, epi):
    """The halo-row pph kernel over 64-px column strips of images wider than 128 px (EDSR at LR 256: the
    body convs, their dgrads and the upsample convs' pixel-shuffled stores): tiles of 4 rows x 64 px, each
    halo row's two border columns DMA'd from the neighbouring strips (zeros at the image edges), the
    epilogue mapping tile rows to pixels -- against float64 on the same bf16 operands (every element within
    two bf16 steps plus 1e-3 of the range) and against the per-tap pp kernel it replaces (variant 77)
    within one bf16 step; 3 and 5 strips, a partial 256-channel tile, the pixel-shuffled store."""
    N, H, W, cin, cout, ps = shape
    torch.manual_seed(41)
    dt = torch.bfloat16
    lib = _lib.load()
    conv = nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    spec = C.ConvSpec(cin, cout, out_ps=ps)
    wf, _, bg = C.prepared(conv.weight, conv.bias, spec, dt)
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    yshape = C._out_shape(spec, N, H, W)
    res = torch.randn(yshape, device=cuda).to(dt) if epi == 'relu_res' and ps == 0 else None
    kw = dict(act=_lib.ACT_RELU) if epi == 'relu_res' else {}
    outs = []
    try:
        for variant in (0, 77):
            _lib.check(lib.sr_conv3x3_set_variant(variant))
            name = lib.sr_conv3x3_fwd_kernel_name(C._desc(dt, N, H, W, cin, cin, cout, cout, cout, out_ps=ps))
            assert (name == b'conv3x3_fwd_pph_kernel') == (variant == 0), (variant, name)
            y = torch.empty(yshape, device=cuda, dtype=dt)
            C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout, out_ps=ps, res=res, **kw)
            outs.append(y)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    torch.cuda.synchronize()
    ref = F.conv2d(x.permute(0, 3, 1, 2).double().cpu(), bf(conv.weight.detach().cpu()).double(),
                   conv.bias.detach().cpu().double(), padding=1)
    if ps:
        ref = F.pixel_shuffle(ref, ps)
    if epi == 'relu_res':
        ref = F.relu(ref)
        if res is not None:
            ref = ref + res.permute(0, 3, 1, 2).double().cpu()
    got = outs[0].permute(0, 3, 1, 2).double().cpu()
    tol = ref.abs() * 2.0 ** -7 + 1e-3 * ref.abs().max().item()
    assert bool(((got - ref).abs() <= tol).all()), (got - ref).abs().max().item()
    _same_or_ulp(outs[0], outs[1], exact=False)


@pytest.mark.parametrize('shape', [(2, 256, 256, 64, 0), (1, 256, 1024, 64, 2), (1, 256, 1024, 128, 2),
                                   (2, 128, 128, 128, 0)])
def test_two_interval_schedule_bitwise(cuda, shape):
    """The two-interval (4 barriers per K-step) schedules of the pph fwd / dgrad kernel and the pp wgrad
    kernel (the default since round 3) keep every accumulator's K order: outputs, pixel-shuffled
    dgrads and weight / bias gradients are bitwise equal to the 4-phase kernels (variant 59)."""
    from basicsr4rs_amd import _lib
    from basicsr4rs_amd.ops import conv as C
    N, cin, cout, hw, ps = shape
    torch.manual_seed(5)
    dt = torch.bfloat16
    conv = torch.nn.Conv2d(cin, cout, 3, 1, 1).to(cuda)
    spec = C.ConvSpec(cin, cout, out_ps=ps)
    x = torch.randn(N, hw, hw, cin, device=cuda).to(dt)
    wf, wd, bg = C.prepared(conv.weight, conv.bias, spec, dt)
    yshape = C._out_shape(spec, N, hw, hw)
    dy = torch.randn(yshape, device=cuda).to(dt)
    lib = _lib.load()

    def run():
        y = torch.empty(yshape, device=cuda, dtype=dt)
        C.conv_fwd_raw(x, wf, bg, y, N, hw, hw, cin, cout, cout, out_ps=ps)
        dx = torch.empty(N, hw, hw, cin, device=cuda, dtype=dt)
        C.conv_fwd_raw(dy, wd, None, dx, N, hw, hw, cout, cin, cin, in_ps=ps, ldx=dy.shape[-1])
        dw, db = C.conv_wgrad_raw(dy, x, N, hw, hw, cin, cin, cout, cout, out_ps=ps)
        return y, dx, dw, db

    ref = run()
    for v in (59, 61):  # 59: 4-phase kernels; 61: pph two-interval without the two-step-ahead B prefetch
        _lib.check(lib.sr_conv3x3_set_variant(v))
        try:
            got = run()
        finally:
            _lib.check(lib.sr_conv3x3_set_variant(0))
        for name, a, b in zip(('y', 'dx', 'dw', 'db'), ref, got):
            assert torch.equal(a, b), (v, name, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize('shape', [(2, 64, 64), (3, 20, 128), (1, 5, 64), (32, 64, 64), (8, 64, 64), (16, 32, 128)])
def test_band_dot_partials(cuda, shape):
    """Band kernel residual + dot epilogue (RCAB conv1 dgrad with the previous block's channel-attention
    dot fused, rcan_arch.py:19-27): y equals the plain residual call bitwise, and the partial rows sum
    per image to sum_p y[n, p, c] * dot[n, p, c] over the stored bf16 y (fp64 reference, fp32 sums) --
    per-row partials and (round 6) partials summed over each band (RCAN B 32: 8 rows per band, 16 partial
    rows per image), whose count the host query reports."""
    N, H, W = shape
    rows = N * H
    rpb = rows // 256 if rows % 256 == 0 and rows >= 512 and H % (rows // 256) == 0 else 0
    lib0 = _lib.load()
    d = C._desc(torch.bfloat16, N, H, W, 64, 64, 64, 64, 64)
    P = lib0.sr_conv3x3_fwd_colsum_parts(d)
    assert P == (H // rpb if rpb else H) * (8 if W == 128 else 4) // 2, (P, rpb)
    cin = cout = 64
    dt = torch.bfloat16
    torch.manual_seed(21)
    lib = _lib.load()
    x = torch.randn(N, H, W, cin, device=cuda).to(dt)
    wf = (torch.randn(cout, 9 * cin, device=cuda) * 0.05).to(dt)
    res = torch.randn(N, H, W, cout, device=cuda).to(dt)
    dot = torch.randn(N, H, W, cout, device=cuda).to(dt)
    assert C.dot_partials_ok(dt, N, H, W, cin, cout)
    y0 = torch.empty(N, H, W, cout, device=cuda, dtype=dt)
    C.conv_fwd_raw(x, wf, None, y0, N, H, W, cin, cout, cout, res=res, beta=1.0)
    y1 = torch.empty_like(y0)
    y1, parts = C.conv_fwd_raw(x, wf, None, y1, N, H, W, cin, cout, cout, res=res, beta=1.0, colsum=True, dot=dot)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert parts.shape == (N, P, cout)
    ref = (y1.double() * dot.double()).sum((1, 2))
    got = parts.double().sum(1)
    scale = (y1.double() * dot.double()).abs().sum((1, 2)).max().item()
    assert (got - ref).abs().max().item() <= 1e-5 * scale
    # not on the band kernel (variant 34: the tile kernel) the dot request fails loudly
    _lib.check(lib.sr_conv3x3_set_variant(34))
    try:
        assert not C.dot_partials_ok(dt, N, H, W, cin, cout)
        with pytest.raises((RuntimeError, ValueError)):  # C status, or no fused sums on that kernel at all
            C.conv_fwd_raw(x, wf, None, y1, N, H, W, cin, cout, cout, res=res, beta=1.0, colsum=True, dot=dot)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))


def test_prepared_images_freed_with_their_weight(cuda):
    """The GEMM-image registry (ops.conv._PREP_ALL) is weak: a discarded weight's images are freed
    (round-3 verdict: the registry held every weight ever prepared for the process lifetime)."""
    import gc
    gc.collect()
    before = set(C._PREP_ALL.keys())
    conv = torch.nn.Conv2d(16, 16, 3, 1, 1).to(cuda)
    spec = C.ConvSpec(16, 16)
    C.prepared(conv.weight, conv.bias, spec, torch.bfloat16)
    new = set(C._PREP_ALL.keys()) - before
    assert len(new) == 1
    del conv
    gc.collect()
    C._retire_table(torch.bfloat16)
    gc.collect()
    # (other tests' discarded weights may be collected here too: only this weight's entry is checked)
    assert not (new & set(C._PREP_ALL.keys()))
