"""Full SR train step on the GPU vs the CPU oracle (sr_model.py:91-118 semantics).

SRModel (HIP forward/backward, fused L1, fused Adam+EMA over the flat parameter vector)
runs 2 fp32 steps of a small EDSR; the oracle replays them on the CPU with the reference's
own optimizer (torch.optim.Adam, base_model.py:107-124) and EMA formula (base_model.py:75-82).
Tolerance: relative 2e-4 on every parameter and EMA parameter after 2 steps.
"""
import copy

import pytest
import torch

from oracle import nets as O

pytestmark = pytest.mark.gpu


def _opt(amp=False, ema=0.999):
    return dict(model_type='SRModel', is_train=True, dist=False, num_gpu=1, path={},
                network_g=dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=2, upscale=4,
                               res_scale=1),
                train=dict(ema_decay=ema, use_amp=amp, optim_g=dict(type='Adam', lr=1e-3, weight_decay=0,
                                                                       betas=[0.9, 0.99]),
                           scheduler=dict(type='MultiStepLR', milestones=[100], gamma=0.5),
                           pixel_opt=dict(type='L1Loss', loss_weight=1.0, reduction='mean')))


def test_sr_model_train_step_matches_oracle(cuda):
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    torch.manual_seed(0)
    model = build_model(_opt())
    net = model.get_bare_model(model.net_g)
    sd0 = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    params = {k: v.clone().requires_grad_(True) for k, v in sd0.items()}
    ema = {k: v.clone() for k, v in sd0.items()}
    opt = torch.optim.Adam(list(params.values()), lr=1e-3, betas=(0.9, 0.99))
    lq = torch.rand(2, 3, 16, 16, generator=torch.Generator().manual_seed(0))
    gt = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    model.feed_data({'lq': lq, 'gt': gt})
    for it in (1, 2):
        model.update_learning_rate(it)
        model.optimize_parameters(it)
        opt.zero_grad()
        loss = O.l1_loss(O.edsr(params, lq, num_block=2, upscale=4), gt)
        loss.backward()
        opt.step()
        with torch.no_grad():
            for k in ema:
                ema[k].mul_(0.999).add_(params[k], alpha=0.001)
        got = model.get_current_log()['l_pix']
        assert abs(got - loss.item()) < 1e-5 * max(1.0, abs(loss.item()))
    for k, v in net.state_dict().items():
        ref = params[k].detach()
        err = (v.cpu() - ref).abs().max().item() / max(1e-3, ref.abs().max().item())
        assert err < 2e-4, (k, err)
    for k, v in model.net_g_ema.state_dict().items():
        err = (v.cpu() - ema[k]).abs().max().item() / max(1e-3, ema[k].abs().max().item())
        assert err < 2e-4, (k, err)
    # optimizer state_dict has torch.optim.Adam's layout
    sd = model.optimizer_g.state_dict()
    assert set(sd['state'][0].keys()) == {'step', 'exp_avg', 'exp_avg_sq'}
    assert float(sd['state'][0]['step']) == 2.0


def test_sr_model_bf16_step_runs(cuda):
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    torch.manual_seed(0)
    model = build_model(_opt(amp=True))
    lq = torch.rand(2, 3, 16, 16)
    gt = torch.rand(2, 3, 64, 64)
    model.feed_data({'lq': lq, 'gt': gt})
    losses = []
    for it in range(1, 6):
        model.optimize_parameters(it)
        losses.append(model.get_current_log()['l_pix'])
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


@pytest.mark.parametrize('amp', [False, True])
def test_sr_model_hip_graph_matches_eager(cuda, amp):
    """train.cuda_graph: steps 1-2 eager, step 3 captured + run, steps 4-6 graph replays (with an
    lr milestone crossing) must give bitwise the same parameters, EMA and losses as eager steps."""
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        o = _opt(amp=amp)
        o['train']['cuda_graph'] = graph
        o['train']['scheduler'] = dict(type='MultiStepLR', milestones=[4], gamma=0.5)
        model = build_model(o)
        losses = []
        for it in range(1, 7):
            g0 = torch.Generator().manual_seed(it)
            model.feed_data({'lq': torch.rand(2, 3, 16, 16, generator=g0), 'gt': torch.rand(2, 3, 64, 64, generator=g0)})
            model.update_learning_rate(it)
            model.optimize_parameters(it)
            losses.append(model.get_current_log()['l_pix'])
        assert (model._graph is not None) == graph
        net = model.get_bare_model(model.net_g)
        runs.append((losses, {k: v.detach().cpu().clone() for k, v in net.state_dict().items()},
                     {k: v.detach().cpu().clone() for k, v in model.net_g_ema.state_dict().items()},
                     float(model.optimizer_g.state_dict()['state'][0]['step'])))
    (l0, p0, e0, s0), (l1, p1, e1, s1) = runs
    assert l0 == l1
    assert s0 == s1 == 6.0
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k
        assert torch.equal(e0[k], e1[k]), k


def test_validation_between_graph_replays(cuda, tmp_path):
    """SRModel.nondist_validation (sr_model.py:183-248 semantics) on PNG pairs of another shape,
    run between HIP-graph replays (train.cuda_graph): the metrics equal PSNR / SSIM of the
    oracle's EMA-net outputs (tensor2img -> calculate_*), the SR images are written, and the
    training that follows is bitwise the eager run's (validation never touches the captured
    step's static inputs)."""
    import numpy as np

    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.data import build_dataloader, build_dataset
    from basicsr4rs_amd.metrics import calculate_psnr, calculate_ssim
    from basicsr4rs_amd.models import build_model
    from basicsr4rs_amd.utils.img_util import tensor2img
    from tests.test_data import _make_pairs
    _make_pairs(tmp_path, 3, 12, 12, 4)
    vopt = dict(name='val', type='PairedImageDataset', dataroot_gt=str(tmp_path / 'gt'),
                dataroot_lq=str(tmp_path / 'lq'), io_backend=dict(type='disk'), scale=4, phase='val')
    vds = build_dataset(vopt)
    vloader = build_dataloader(vds, vopt)
    metrics = dict(psnr=dict(type='calculate_psnr', crop_border=4, test_y_channel=False),
                   ssim=dict(type='calculate_ssim', crop_border=4, test_y_channel=False))
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        o = _opt()
        o['train']['cuda_graph'] = graph
        o['val'] = dict(metrics=metrics)
        o['path'] = dict(visualization=str(tmp_path / f'vis{int(graph)}'))
        model = build_model(o)
        losses = []
        for it in range(1, 7):
            g0 = torch.Generator().manual_seed(it)
            model.feed_data({'lq': torch.rand(2, 3, 16, 16, generator=g0), 'gt': torch.rand(2, 3, 64, 64, generator=g0)})
            model.update_learning_rate(it)
            model.optimize_parameters(it)
            losses.append(model.get_current_log()['l_pix'])
            if graph and it == 4:
                assert model._graph is not None
                ema_sd = {k: v.detach().cpu().clone() for k, v in model.net_g_ema.state_dict().items()}
                model.validation(vloader, it, None, save_img=True)
                got = dict(model.metric_results)
                exp = {'psnr': [], 'ssim': []}
                for i in range(len(vds)):
                    d = vds[i]
                    sr = tensor2img([O.edsr(ema_sd, d['lq'][None], num_block=2, upscale=4)])
                    hr = tensor2img([d['gt'][None]])
                    exp['psnr'].append(calculate_psnr(sr, hr, 4))
                    exp['ssim'].append(calculate_ssim(sr, hr, 4))
                assert abs(got['psnr'] - np.mean(exp['psnr'])) < 0.05, (got, exp)
                assert abs(got['ssim'] - np.mean(exp['ssim'])) < 1e-3, (got, exp)
                assert model.best_metric_results['val']['psnr']['iter'] == it
                assert len(list((tmp_path / 'vis1').rglob('*_4.png'))) == 3
        net = model.get_bare_model(model.net_g)
        runs.append((losses, {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}))
    (l0, p0), (l1, p1) = runs
    assert l0 == l1
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k


_NETS = {
    'edsr': dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=2, upscale=4, res_scale=1),
    'rcan': dict(type='RCAN', num_in_ch=3, num_out_ch=3, num_feat=64, num_group=2, num_block=2, squeeze_factor=16,
                 upscale=4, res_scale=1),
    'rrdb': dict(type='RRDBNet', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=2, num_grow_ch=32, scale=4),
    'swinir': dict(type='SwinIR', upscale=4, in_chans=3, img_size=16, window_size=8, img_range=1., depths=[2, 2],
                   embed_dim=60, num_heads=[6, 6], mlp_ratio=2, upsampler='pixelshuffle', resi_connection='1conv'),
}


@pytest.mark.parametrize('net', ['rcan', 'swinir', 'edsr', 'rrdb'])
def test_async_wgrad_delayed_side_stream_bitwise(cuda, net):
    """The side stream held back by a spin kernel queued ahead of each backward: the main stream then
    runs the whole dgrad chain, including autograd's accumulation of a residual's two gradient
    contributions, before any side-stream weight gradient reads its dy.  That accumulation would be
    done IN PLACE into a dy the side stream still has to read (RCAN body conv, SwinIR RSTB conv:
    round-3 finding, nondeterministic SwinIR runs) unless the dy stays referenced until the join
    (ops.conv._ASYNC['hold']); losses and parameters must equal the single-stream run bitwise."""
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    from basicsr4rs_amd.ops import conv as C
    runs = []
    for use_async in (False, True):
        torch.manual_seed(0)
        opt = _opt(amp=True)
        opt['network_g'] = dict(_NETS[net])
        opt['train']['cuda_graph'] = False
        opt['train']['async_wgrad'] = use_async
        model = build_model(opt)
        lq = torch.rand(4, 3, 16, 16, generator=torch.Generator().manual_seed(0)).to(cuda)
        gt = torch.rand(4, 3, 64, 64, generator=torch.Generator().manual_seed(1)).to(cuda)
        model.feed_data({'lq': lq, 'gt': gt})
        losses = []
        for it in range(1, 4):
            model.update_learning_rate(it)
            if use_async:
                with torch.cuda.stream(C._side_stream(torch.device(cuda))):
                    torch.cuda._sleep(20_000_000)
            model.optimize_parameters(it)
            losses.append(model.get_current_log()['l_pix'])
        torch.cuda.synchronize()
        net_ = model.get_bare_model(model.net_g)
        runs.append((losses, {k: v.detach().clone() for k, v in net_.state_dict().items()}))
    assert runs[0][0] == runs[1][0]
    for k in runs[0][1]:
        assert torch.equal(runs[0][1][k], runs[1][1][k]), k


@pytest.mark.parametrize('net', sorted(_NETS))
@pytest.mark.parametrize('graph', [False, True])
def test_async_wgrad_bitwise_equals_sync(cuda, net, graph):
    """Weight gradients on the side stream (train.async_wgrad, ops.conv.async_wgrad) give bitwise the same
    losses, parameters and EMA as the single-stream order, eager and HIP-graph captured (eager
    steps 1-2, capture at 3, replays 4-5): the kernels and their inputs are the same, only the
    stream they run on differs -- so any missing fork / join / record_stream shows up here."""
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    runs = []
    for use_async in (False, True, 'reduce'):
        torch.manual_seed(0)
        opt = _opt(amp=True)
        opt['network_g'] = dict(_NETS[net])
        opt['train']['cuda_graph'] = graph
        opt['train']['async_wgrad'] = use_async
        model = build_model(opt)
        lq = torch.rand(4, 3, 16, 16, generator=torch.Generator().manual_seed(0)).to(cuda)
        gt = torch.rand(4, 3, 64, 64, generator=torch.Generator().manual_seed(1)).to(cuda)
        model.feed_data({'lq': lq, 'gt': gt})
        losses = []
        for it in range(1, 6):
            model.update_learning_rate(it)
            model.optimize_parameters(it)
            losses.append(model.get_current_log()['l_pix'])
        assert model.async_wgrad == use_async
        assert (model._graph is not None) == graph
        net_ = model.get_bare_model(model.net_g)
        runs.append((losses, {k: v.detach().clone() for k, v in net_.state_dict().items()},
                     {k: v.detach().clone() for k, v in model.net_g_ema.state_dict().items()}))
    (l0, s0, e0) = runs[0]
    for (l1, s1, e1) in runs[1:]:  # whole weight gradients / only their reduces on the side stream
        assert l0 == l1
        for k in s0:
            assert torch.equal(s0[k], s1[k]), k
            assert torch.equal(e0[k], e1[k]), k
