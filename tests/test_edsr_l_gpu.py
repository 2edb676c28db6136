"""The headline config C2 at net level: EDSR_Lx4 (num_feat 256, num_block 32, res_scale 0.1,
upscale 4; basicsr/archs/edsr_arch.py:30-61, options/train/EDSR/train_EDSR_Lx4.yml:43-52).

* fp32 (exact-f32 MFMA path) at 1x3x48x48 against the CPU oracle run in float64: output max
  |err| <= 1e-3 (north_star's bar) and every parameter gradient within 1e-3 of its max
  magnitude (observed: 4e-7 / 3e-6).  The oracle's own fp32 CPU backward is the noisier side
  here: torch-CPU's fp32 conv backward is 5e-3 off float64 on body.17.conv1 (tools/diag_edsr_l.py),
  so float64 is the reference;
* bf16 (autocast, the bench's precision) against the oracle evaluated in fp32 on the same
  bf16-rounded weights and input (the bf16 kernels round every activation, the oracle does not);
* one full-size B = 32 train step (64x64 -> 256x256, bf16, HIP graph): finite loss, every
  parameter and EMA parameter moved, and graph replays bitwise equal to eager steps.
"""
import copy
import math

import pytest
import torch

from oracle import nets as O

pytestmark = pytest.mark.gpu

EDSR_L = dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=256, num_block=32, upscale=4, res_scale=0.1,
              img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])


def _oracle(sd, x):
    return O.edsr(sd, x, num_block=32, upscale=4, res_scale=0.1)


def test_edsr_l_fp32_forward_and_grads(cuda):
    from basicsr4rs_amd.archs import build_network
    torch.manual_seed(0)
    net = build_network(dict(EDSR_L))
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    x = torch.rand(1, 3, 48, 48, generator=torch.Generator().manual_seed(1))
    sdg = {k: v.clone().double().requires_grad_(True) for k, v in sd.items()}
    ref = _oracle(sdg, x.double())
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    (ref * g).sum().backward()
    gn = copy.deepcopy(net).to(cuda)
    out = gn(x.to(cuda))
    assert out.shape == (1, 3, 192, 192)
    err = (out.detach().cpu().double() - ref.detach()).abs().max().item()
    assert err <= 1e-3, err
    (out * g.float().to(cuda)).sum().backward()
    worst = 0.0
    for n, p in gn.named_parameters():
        r = sdg[n].grad
        e = (p.grad.cpu().double() - r).abs().max().item() / max(1e-6, r.abs().max().item())
        worst = max(worst, e)
        assert e <= 1e-3, (n, e)
    print(f'EDSR_Lx4 fp32: out max|err| {err:.3e}, worst relative param-grad err {worst:.3e}')


def test_edsr_l_bf16_forward(cuda):
    from basicsr4rs_amd.archs import build_network
    torch.manual_seed(0)
    net = build_network(dict(EDSR_L))
    sd = {k: v.detach().to(torch.bfloat16).float() for k, v in net.state_dict().items()}  # bf16-rounded weights
    net.load_state_dict(sd)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    xr = x.to(torch.bfloat16).float()
    ref = _oracle(sd, xr)
    gn = copy.deepcopy(net).to(cuda)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = gn(x.to(cuda))
    d = out.float().cpu() - ref
    mse = (d**2).mean().item()
    psnr = 10 * math.log10(1.0 / mse)
    print(f'EDSR_Lx4 bf16: max|err| {d.abs().max().item():.3e}, PSNR vs fp32 oracle {psnr:.2f} dB')
    assert d.abs().max().item() < 5e-3  # observed 1.2e-3
    assert psnr > 65.0  # observed 72.2 dB


def _opt(graph):
    return dict(model_type='SRModel', is_train=True, dist=False, num_gpu=1, path={}, network_g=dict(EDSR_L),
                train=dict(ema_decay=0.999, use_amp=True, cuda_graph=graph,
                           optim_g=dict(type='Adam', lr=1e-4, weight_decay=0, betas=[0.9, 0.99]),
                           scheduler=dict(type='MultiStepLR', milestones=[200000], gamma=0.5),
                           pixel_opt=dict(type='L1Loss', loss_weight=1.0, reduction='mean')))


def test_edsr_l_full_size_graph_step(cuda):
    """B = 32, 64x64 -> 256x256 bf16 (the bench workload): eager steps 1-2, capture at 3, replay
    4; the same 4 steps eager must give bitwise the same parameters, EMA and losses."""
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    lq = torch.rand(32, 3, 64, 64, generator=torch.Generator(device=cuda).manual_seed(0), device=cuda)
    gt = torch.rand(32, 3, 256, 256, generator=torch.Generator(device=cuda).manual_seed(1), device=cuda)
    runs = []
    for graph in (False, True):
        torch.manual_seed(42)
        model = build_model(_opt(graph))
        net = model.get_bare_model(model.net_g)
        p0 = {k: v.detach().clone() for k, v in net.state_dict().items()}
        model.feed_data({'lq': lq, 'gt': gt})
        losses = []
        for it in range(1, 5):
            model.update_learning_rate(it)
            model.optimize_parameters(it)
            losses.append(model.get_current_log()['l_pix'])
        assert (model._graph is not None) == graph
        assert all(math.isfinite(v) for v in losses), losses
        sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
        ema = {k: v.detach().clone() for k, v in model.net_g_ema.state_dict().items()}
        for k in p0:
            assert not torch.equal(sd[k], p0[k]), f'{k} did not change'
            assert not torch.equal(ema[k], p0[k]), f'EMA {k} did not change'
        runs.append((losses, sd, ema))
        del model
        torch.cuda.empty_cache()
    (l0, s0, e0), (l1, s1, e1) = runs
    assert l0 == l1
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
        assert torch.equal(e0[k], e1[k]), k
