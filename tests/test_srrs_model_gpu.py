"""SRRSModel / SwinIRRSModel (basicsr/models/srrs_model.py:33-88, swinir_model.py:40-42): the AMP
train step of the fork's remote-sensing configs (options/train/SwinIR/train_SwinIR_S2N256_scratch.yml
selects SwinIRRSModel).

* fp32 (use_amp false): two steps replayed by the CPU oracle with torch.optim.Adam and the EMA
  formula, relative 2e-4 (as the SRModel test);
* bf16 autocast (use_amp true; the reference's fp16 + GradScaler, bf16 here needs no scaler): the
  step's loss is the oracle's fp32 loss on the same weights within 1e-2 relative, and the parameter
  update it applies points the same way as the oracle's fp32 Adam update (cosine >= 0.98 over all
  parameters; Adam's first step is ~lr * sign(g), so bf16 rounding flips only the signs of
  near-zero gradient entries);
* the NaN / Inf branch: a non-finite loss skips the optimizer step (parameters, EMA and the Adam
  step count untouched, gradients zero, the batch dropped) and training continues afterwards.
"""
import pytest
import torch

from oracle import nets as O

pytestmark = pytest.mark.gpu

EDSR = dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=2, upscale=4, res_scale=1)
SWINIR = dict(type='SwinIR', upscale=4, in_chans=3, img_size=16, window_size=8, img_range=1., depths=[2],
              embed_dim=60, num_heads=[6], mlp_ratio=2, upsampler='pixelshuffle', resi_connection='1conv',
              drop_path_rate=0.)


def _opt(model_type, net, amp):
    return dict(model_type=model_type, is_train=True, dist=False, num_gpu=1, path={}, network_g=dict(net), scale=4,
                train=dict(ema_decay=0.999, use_amp=amp,
                           optim_g=dict(type='Adam', lr=1e-3, weight_decay=0, betas=[0.9, 0.99]),
                           scheduler=dict(type='MultiStepLR', milestones=[100], gamma=0.5),
                           pixel_opt=dict(type='L1Loss', loss_weight=1.0, reduction='mean')))


def _oracle(net, sd, lq):
    if net['type'] == 'EDSR':
        return O.edsr(sd, lq, num_block=2, upscale=4)
    return O.swinir(sd, lq, net)


def _replay(net, sd0, lq, gt, steps):
    params = {k: v.clone().requires_grad_(True) for k, v in sd0.items() if v.is_floating_point()}
    ema = {k: v.clone() for k, v in params.items()}
    opt = torch.optim.Adam(list(params.values()), lr=1e-3, betas=(0.9, 0.99))
    losses = []
    for _ in range(steps):
        opt.zero_grad()
        full = dict(sd0, **params)
        loss = O.l1_loss(_oracle(net, full, lq), gt)
        loss.backward()
        opt.step()
        with torch.no_grad():
            for k in ema:
                ema[k].mul_(0.999).add_(params[k], alpha=0.001)
        losses.append(loss.item())
    return params, ema, losses


@pytest.mark.parametrize('mtype,net', [('SRRSModel', EDSR), ('SwinIRRSModel', SWINIR)])
def test_srrs_fp32_steps_match_oracle(cuda, mtype, net):
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    torch.manual_seed(0)
    model = build_model(_opt(mtype, net, amp=False))
    assert type(model).__name__ == mtype
    bare = model.get_bare_model(model.net_g)
    sd0 = {k: v.detach().cpu().clone() for k, v in bare.state_dict().items()}
    lq = torch.rand(2, 3, 16, 16, generator=torch.Generator().manual_seed(0))
    gt = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    got = []
    for it in (1, 2):
        model.feed_data({'lq': lq, 'gt': gt})
        model.update_learning_rate(it)
        model.optimize_parameters(it)
        got.append(model.get_current_log()['l_pix'])
    params, ema, losses = _replay(net, sd0, lq, gt, 2)
    for a, b in zip(got, losses):
        assert abs(a - b) < 1e-5 * max(1.0, abs(b)), (got, losses)
    for k, v in bare.state_dict().items():
        if k in params:
            err = (v.cpu() - params[k].detach()).abs().max().item() / max(1e-3, params[k].abs().max().item())
            assert err < 2e-4, (k, err)
    for k, v in model.net_g_ema.state_dict().items():
        if k in ema:
            err = (v.cpu() - ema[k]).abs().max().item() / max(1e-3, ema[k].abs().max().item())
            assert err < 2e-4, (k, err)


@pytest.mark.parametrize('mtype,net', [('SRRSModel', EDSR), ('SwinIRRSModel', SWINIR)])
def test_srrs_bf16_step_and_nan_skip(cuda, mtype, net):
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    torch.manual_seed(0)
    model = build_model(_opt(mtype, net, amp=True))
    bare = model.get_bare_model(model.net_g)
    sd0 = {k: v.detach().cpu().clone() for k, v in bare.state_dict().items()}
    lq = torch.rand(2, 3, 16, 16, generator=torch.Generator().manual_seed(0))
    gt = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))

    # a NaN batch first: skipped, nothing moves
    bad = lq.clone()
    bad[0, 0, 3, 3] = float('nan')
    model.feed_data({'lq': bad, 'gt': gt})
    model.update_learning_rate(1)
    model.optimize_parameters(1)
    assert not hasattr(model, 'lq') and not hasattr(model, 'output')
    assert model.optimizer_g.nstep == 0
    assert float(model.flat_g.grad.abs().max()) == 0.0
    for k, v in bare.state_dict().items():
        assert torch.equal(v.cpu(), sd0[k]), k
    for k, v in model.net_g_ema.state_dict().items():
        assert torch.equal(v.cpu(), sd0[k]), k

    # then a real bf16 step
    model.feed_data({'lq': lq, 'gt': gt})
    model.update_learning_rate(2)
    model.optimize_parameters(2)
    loss = model.get_current_log()['l_pix']
    assert model.optimizer_g.nstep == 1
    params, _, losses = _replay(net, sd0, lq, gt, 1)
    assert abs(loss - losses[0]) < 1e-2 * abs(losses[0]), (loss, losses)
    d_gpu = torch.cat([(v.cpu() - sd0[k]).reshape(-1) for k, v in bare.state_dict().items() if k in params])
    d_ref = torch.cat([(params[k].detach() - sd0[k]).reshape(-1) for k in bare.state_dict() if k in params])
    cos = torch.nn.functional.cosine_similarity(d_gpu.double(), d_ref.double(), dim=0).item()
    print(f'{mtype} bf16: loss {loss:.6f} vs oracle fp32 {losses[0]:.6f}, update cosine {cos:.4f}')
    assert cos >= 0.98, cos


class _ValSet(torch.utils.data.Dataset):
    """Two 4-band [-1, 1] LR / GT pairs (a 16x16 and a 12x12 LR tile: the second is padded to the
    window by SwinIRModel.test) with reference-style paths."""

    def __init__(self):
        self.opt = {'name': 'S2N_val'}
        g = torch.Generator().manual_seed(11)
        self.items = []
        for i, hw in enumerate((16, 12)):
            lq = torch.rand(4, hw, hw, generator=g) * 2.2 - 1.1
            gt = torch.rand(4, 4 * hw, 4 * hw, generator=g) * 2 - 1
            self.items.append({'lq': lq, 'gt': gt, 'lq_path': f'val/lq/tile_{i}.png'})

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def test_swinirrs_validation_minusone_one(cuda, tmp_path):
    """SwinIRRSModel validation on [-1, 1] 4-band tensors (basicsr/models/srrs_model.py:93-138,
    basicsr/utils/img_util.py:99-128): per-image PSNR / SSIM on the clamp / (x + 1) / 2 / uint8
    images equal the oracle's (net forward restated on the CPU in fp32, SwinIRModel.test's reflect
    pad and crop, oracle/metrics.py conversion and PSNR) within 0.05 dB; the averages, the per-image
    CSV and the RGB / NIR images land where the reference writes them."""
    import csv
    import os

    import numpy as np
    from torch.nn import functional as F

    from basicsr4rs_amd.models import build_model
    from oracle import metrics as OM
    net = dict(SWINIR, in_chans=4)
    opt = _opt('SwinIRRSModel', net, amp=False)
    opt['name'] = 'rs_val'
    opt['path'] = {'visualization': str(tmp_path / 'vis')}
    opt['val'] = {'metrics': {'psnr': {'type': 'calculate_psnr', 'crop_border': 4, 'test_y_channel': False},
                              'ssim': {'type': 'calculate_ssim', 'crop_border': 4, 'test_y_channel': False}}}
    torch.manual_seed(0)
    model = build_model(opt)
    sd = {k: v.detach().cpu().clone() for k, v in model.net_g_ema.state_dict().items()}
    ds = _ValSet()
    loader = torch.utils.data.DataLoader(ds, batch_size=1)
    model.validation(loader, 7, None, save_img=True)

    ref_psnr = []
    for it in ds.items:
        lq = it['lq'][None]
        h = lq.shape[-1]
        pad = (8 - h % 8) % 8
        x = F.pad(lq, (0, pad, 0, pad), 'reflect')
        with torch.no_grad():
            out = _oracle(net, sd, x)[:, :, :4 * h, :4 * h]
        ref_psnr.append(OM.psnr(OM.minusone_one_to_ubyte(out.numpy()),
                                OM.minusone_one_to_ubyte(it['gt'][None].numpy()), 4))
    rows = list(csv.reader(open(tmp_path / 'vis' / 'S2N_val_7.csv')))
    assert rows[0] == ['', 'psnr', 'ssim']
    assert [r[0] for r in rows[1:]] == ['val/lq/tile_0', 'val/lq/tile_1']  # srrs_model.py:150-152
    got = [float(r[1]) for r in rows[1:]]
    print('validation psnr', got, 'oracle', ref_psnr)
    assert np.allclose(got, ref_psnr, atol=0.05), (got, ref_psnr)
    assert abs(model.metric_results['psnr'] - float(np.mean(ref_psnr))) < 0.05
    assert all(0.0 < float(r[2]) <= 1.0 for r in rows[1:])
    for key in ('lq', 'gt', 'sr_7'):
        assert os.path.exists(tmp_path / 'vis' / 'RGB' / 'S2N_val' / 'val/lq/tile_0' / f'{key}.png')
        assert os.path.exists(tmp_path / 'vis' / 'NIR' / 'S2N_val' / 'val/lq/tile_1' / f'{key}.png')
    assert not os.path.exists(tmp_path / 'vis' / 'RGB' / 'S2N_val' / 'val/lq/tile_0' / 'sr.png')


def test_swinir_four_band_forward_fp32(cuda):
    """The 4-band (RGB + NIR) SwinIR of the remote-sensing configs (in_chans 4: zero mean,
    swinir_arch.py:750-754) in fp32 against the oracle, on [-1, 1] inputs, direct and through
    SwinIRModel.test's reflect pad (a 12 x 12 LR tile)."""
    from torch.nn import functional as F

    from basicsr4rs_amd.archs import build_network
    net = dict(SWINIR, in_chans=4)
    torch.manual_seed(0)
    g = build_network(dict(net)).eval()
    sd = {k: v.detach().clone() for k, v in g.state_dict().items()}
    gen = torch.Generator().manual_seed(5)
    for hw in (16, 12):
        lq = torch.rand(1, 4, hw, hw, generator=gen) * 2.2 - 1.1
        pad = (8 - hw % 8) % 8
        x = F.pad(lq, (0, pad, 0, pad), 'reflect')
        with torch.no_grad():
            ref = _oracle(net, sd, x)
            out = g.to(cuda)(x.to(cuda)).cpu()
        err = (out - ref).abs().max().item()
        print(f'SwinIR 4-band fp32 {hw}x{hw}: max-abs {err:.2e}, out range {ref.abs().max().item():.3f}')
        assert err <= 1e-3
