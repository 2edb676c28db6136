"""Parity on a real image: the reference's own test image (test_scripts/data/baboon.png, cropped and
x4-box-downsampled into tests/golden/baboon_x4.npz by tests/golden/make_baboon.py) instead of U[0,1)
noise, so the mean shift / img_range 255 arithmetic (basicsr/archs/edsr_arch.py:51-59,
rcan_arch.py:125-133) and the SwinIR window attention see real-image statistics.

* EDSR_M (C1: 4 ResidualBlockNoBN, nf 64, x4) in fp32: output within the north-star bar (max-abs
  1e-3) of the CPU oracle, every parameter gradient of an L1 loss against the real HR crop within
  1e-3 relative;
* RCAN (2 groups x 2 RCAB) and SwinIR (embed 60, depths [2, 2]) fp32 forward within 1e-3;
* EDSR_M in bf16 autocast: PSNR against the fp32 oracle above 50 dB.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import nets as O

HERE = os.path.dirname(os.path.abspath(__file__))


def _tile():
    d = np.load(os.path.join(HERE, 'golden', 'baboon_x4.npz'))
    lr = torch.from_numpy(d['lr']).permute(2, 0, 1)[None].float() / 255.
    hr = torch.from_numpy(d['hr']).permute(2, 0, 1)[None].float() / 255.
    return lr, hr


def test_baboon_fixture_consistent():
    """The fixture is what its generator says: HR 256^2 uint8, LR = rounded 4x4 box mean of it."""
    d = np.load(os.path.join(HERE, 'golden', 'baboon_x4.npz'))
    hr, lr = d['hr'], d['lr']
    assert hr.shape == (256, 256, 3) and lr.shape == (64, 64, 3) and hr.dtype == lr.dtype == np.uint8
    box = np.clip(np.rint(hr.reshape(64, 4, 64, 4, 3).astype(np.float64).mean(axis=(1, 3))), 0, 255)
    assert np.array_equal(box.astype(np.uint8), lr)
    assert 40 < hr.std() < 90  # a textured natural image, not a flat or noise tile


EDSR_M = dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=4, upscale=4, res_scale=1,
              img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])
RCAN_S = dict(type='RCAN', num_in_ch=3, num_out_ch=3, num_feat=64, num_group=2, num_block=2, squeeze_factor=16,
              upscale=4, res_scale=1, img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])
SWINIR_S = dict(type='SwinIR', upscale=4, in_chans=3, img_size=64, window_size=8, img_range=1., depths=[2, 2],
                embed_dim=60, num_heads=[6, 6], mlp_ratio=2, upsampler='pixelshuffle', resi_connection='1conv')


def _oracle(cfg, sd, x):
    if cfg['type'] == 'EDSR':
        return O.edsr(sd, x, num_block=cfg['num_block'], upscale=4, res_scale=cfg['res_scale'])
    if cfg['type'] == 'RCAN':
        return O.rcan(sd, x, num_group=cfg['num_group'], num_block=cfg['num_block'], upscale=4)
    return O.swinir(sd, x, cfg)


@pytest.mark.gpu
def test_edsr_m_real_image_fp32_fwd_bwd(cuda):
    from basicsr4rs_amd.archs import build_network
    lr, hr = _tile()
    torch.manual_seed(42)
    net = build_network(dict(EDSR_M))
    sd = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in net.state_dict().items()}
    ref = _oracle(EDSR_M, sd, lr)
    O.l1_loss(ref, hr).backward()
    gn = net.to(cuda)
    out = gn(lr.to(cuda))
    (out - hr.to(cuda)).abs().mean().backward()
    err = (out.detach().cpu() - ref.detach()).abs().max().item()
    psnr = 10 * math.log10(1.0 / max(1e-30, ((out.detach().cpu() - ref.detach())**2).mean().item()))
    worst = max(((p.grad.cpu() - sd[n].grad).abs().max().item() / max(1e-12, sd[n].grad.abs().max().item()), n)
                for n, p in gn.named_parameters())
    print(f'EDSR_M fp32 on baboon: max-abs {err:.2e}, PSNR vs oracle {psnr:.1f} dB; worst grad rel err {worst}')
    assert err <= 1e-3
    assert worst[0] <= 1e-3, worst


@pytest.mark.gpu
@pytest.mark.parametrize('cfg', [RCAN_S, SWINIR_S], ids=['rcan', 'swinir'])
def test_real_image_fp32_forward(cuda, cfg):
    from basicsr4rs_amd.archs import build_network
    lr, _ = _tile()
    torch.manual_seed(42)
    net = build_network(dict(cfg)).eval()
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    with torch.no_grad():
        ref = _oracle(cfg, sd, lr)
        out = net.to(cuda)(lr.to(cuda)).cpu()
    err = (out - ref).abs().max().item()
    print(f"{cfg['type']} fp32 on baboon: max-abs {err:.2e}")
    assert err <= 1e-3


@pytest.mark.gpu
def test_edsr_m_real_image_bf16_psnr(cuda):
    from basicsr4rs_amd.archs import build_network
    lr, _ = _tile()
    torch.manual_seed(42)
    net = build_network(dict(EDSR_M)).eval()
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    with torch.no_grad():
        ref = _oracle(EDSR_M, sd, lr)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = net.to(cuda)(lr.to(cuda)).float().cpu()
    psnr = 10 * math.log10(1.0 / max(1e-30, ((out - ref)**2).mean().item()))
    print(f'EDSR_M bf16 on baboon: PSNR vs fp32 oracle {psnr:.1f} dB')
    assert psnr > 50.0
