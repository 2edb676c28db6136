"""The production bf16 kernels inside each benchmarked net, at the benchmark's LR tile.

The other net-level tests run small tiles (16x16) at which the row-streaming kernels are not
selected.  Here each BASELINE workload net runs at reduced depth but at its workload tile, so the
kernels its benchmarked step spends its time in are the ones under test:

* RCAN (nf 64, squeeze 16, 2 groups x 2 RCAB) at 64x64 LR (C3, basicsr/archs/rcan_arch.py:71-135):
  band fwd / dgrad, ring wgrad, pph upsample convs, HR tail conv;
* RRDBNet (nf 64, gc 32, 2 RRDB) at 128x128 LR (C5, rrdbnet_arch.py:66-119): band (+ sliced band
  dgrads), halo, ring wgrad, HR tail;
* EDSR_Lx4 (nf 256, res_scale 0.1, 4 blocks) at 64x64 (C2, edsr_arch.py:30-61): pph fwd and
  pixel-shuffled pph dgrads, pp wgrad with the fused / grouped bias, HR tail -- forward AND backward;
* SwinIR-M geometry (embed 180, 6 heads, window 8, depths [2, 2]) at 64x64 (C4,
  swinir_arch.py:693-933): lin (+ LayerNorm prologue), window attention fwd / bwd, pp wgrads.

Method (each net): weights and input rounded to bf16, the CPU oracle (oracle/nets.py) run in
float64 on them, forward and backward under a fixed random HR output gradient; the HIP net in bf16
autocast on the same values.  Checked: output max error relative to the output range, PSNR, and for
EVERY parameter gradient the cosine to the oracle's (>= 0.995) and the max error relative to its max
magnitude (bound per net, below).  ``ktrace`` records the kernel of every conv / linear / attention
launch; the test asserts the production kernels ran.

Tolerances: bf16 keeps 8 mantissa bits, so every stored activation and gradient carries a relative
rounding error up to 2^-9.  The per-parameter max-error bounds are ~2x the maxima observed in round 4
(printed by each test; profiles/r04/tests): RCAN B 8 0.062 -> 0.12, RCAN B 32 0.036 -> 0.07, EDSR
0.068 -> 0.13; RRDB (0.105) and SwinIR (0.117) keep 0.15 (~1.4x) -- their worst tensors are biases
of 32-channel convs / the qkv weight, whose gradients sum many bf16-rounded terms (SwinIR, round 6: 0.15
/ 0.105 = 1.1x / 1.3x the float64 oracle's own error under emulated bf16 storage,
test_swinir_grad_error_is_bf16_storage_rounding).  Round 5 adds the
per-parameter relative L2 error ||g - g_ref|| / ||g_ref|| at ~1.5x its observed maximum (RCAN B 8
0.049, B 32 0.039, RRDB 0.075, EDSR 0.056, SwinIR 0.097 on a LayerNorm weight): the worst tensors
are short vectors (biases, LayerNorm weights), so it sits close to the max error.  A defect in a kernel (a wrong tap, a missed row, a race) shows up as a
cosine far below 0.99 on the affected tensors, not as a few percent of max error.

``test_rrdb_full_depth_error_is_bf16_storage_rounding`` explains the bench's RRDB bf16 parity
(max-abs 0.0255 / 46.1 dB at 23 RRDB, profiles/r02/bench_rrdb.json): the oracle run with bf16
storage rounding emulated (oracle.nets.bf16_storage) lands at the same error level.
"""
import math

import pytest
import torch

from oracle import nets as O

pytestmark = pytest.mark.gpu

RCAN = dict(type='RCAN', num_in_ch=3, num_out_ch=3, num_feat=64, num_group=2, num_block=2, squeeze_factor=16,
            upscale=4, res_scale=1, img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])
RRDB = dict(type='RRDBNet', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=2, num_grow_ch=32, scale=4)
EDSR_L4 = dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=256, num_block=4, upscale=4, res_scale=0.1,
               img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])
SWINIR_M2 = dict(type='SwinIR', upscale=4, in_chans=3, img_size=64, window_size=8, img_range=1., depths=[2, 2],
                 embed_dim=180, num_heads=[6, 6], mlp_ratio=2, upsampler='pixelshuffle', resi_connection='1conv',
                 drop_path_rate=0.)


def _oracle(cfg):
    t = cfg['type']
    if t == 'RCAN':
        return lambda sd, x: O.rcan(sd, x, num_group=cfg['num_group'], num_block=cfg['num_block'], upscale=4)
    if t == 'RRDBNet':
        return lambda sd, x: O.rrdbnet(sd, x, scale=4, num_block=cfg['num_block'])
    if t == 'EDSR':
        return lambda sd, x: O.edsr(sd, x, num_block=cfg['num_block'], upscale=4, res_scale=cfg['res_scale'])
    return lambda sd, x: O.swinir(sd, x, cfg)


def _bf16_round(t):
    return t.to(torch.bfloat16).float() if t.is_floating_point() else t


def _run(cuda, cfg, batch, lr_px, kernels, out_tol, grad_tol, cos_min=0.995, seed=0, l2_tol=0.08, absent=()):
    from basicsr4rs_amd.archs import build_network
    from basicsr4rs_amd.utils import ktrace
    torch.manual_seed(seed)
    net = build_network(dict(cfg))
    sd = {k: _bf16_round(v.detach()) for k, v in net.state_dict().items()}
    net.load_state_dict(sd)
    x = _bf16_round(torch.rand(batch, 3, lr_px, lr_px, generator=torch.Generator().manual_seed(seed + 1)))
    sdg = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
    ref = _oracle(cfg)(sdg, x.double())
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(seed + 2), dtype=torch.float64)
    (ref * g).sum().backward()
    gn = net.to(cuda)
    ktrace.start()
    try:
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = gn(x.to(cuda))
        (out.float() * g.float().to(cuda)).sum().backward()
    finally:
        stats = ktrace.stop()
    ran = set(stats)
    missing = [k for k in kernels if k not in ran]
    assert not missing, f'production kernels not selected: {missing}; ran {sorted(ran)}'
    assert not ran & set(absent), f'replaced kernels still selected: {sorted(ran & set(absent))}'
    rng = max(1.0, ref.abs().max().item())
    d = out.float().detach().cpu().double() - ref.detach()
    err = d.abs().max().item() / rng
    psnr = 10 * math.log10(rng**2 / max(1e-30, (d**2).mean().item()))
    worst, worst_cos, worst_l2 = (0.0, ''), (1.0, ''), (0.0, '')
    for n, p in gn.named_parameters():
        r = sdg[n].grad
        a = p.grad.detach().cpu().double()
        e = (a - r).abs().max().item() / max(1e-12, r.abs().max().item())
        l2 = (a - r).norm().item() / max(1e-12, r.norm().item())
        cos = torch.nn.functional.cosine_similarity(a.flatten(), r.flatten(), dim=0).item()
        worst, worst_cos, worst_l2 = max(worst, (e, n)), min(worst_cos, (cos, n)), max(worst_l2, (l2, n))
    print(f"{cfg['type']} bf16 B{batch} {lr_px}x{lr_px}: out max err {err:.3e} of range, PSNR {psnr:.1f} dB; "
          f"worst param-grad err {worst[0]:.3e} ({worst[1]}), worst relative L2 {worst_l2[0]:.3e} ({worst_l2[1]}), "
          f"lowest cosine {worst_cos[0]:.5f} ({worst_cos[1]}); kernels {sorted(ran)}")
    assert err <= out_tol, err
    assert worst_cos[0] >= cos_min, worst_cos
    assert worst[0] <= grad_tol, worst
    assert worst_l2[0] <= l2_tol, worst_l2
    return stats


# measured (round 6): worst GPU / emulated ratio 1.295 (relative L2), 1.63 (max error: one element of a
# tensor, the noisier metric); worst emulated error 0.081 (L2) / 0.136 (max)
L2_RATIO, MAX_RATIO = 1.3, 1.8


def test_swinir_grad_error_is_bf16_storage_rounding(cuda):
    """SwinIR-M geometry (2 RSTB x 2 STB, embed 180) at the C4 tile, bf16: every parameter gradient's
    error against the exact float64 oracle is the error the oracle itself shows once the engine's bf16
    storage is emulated (oracle.nets.bf16_storage(grads=True): every stored activation AND gradient
    map rounded to bf16, the attention probabilities forward and the score gradient backward, the MLP
    pre-activation gradient and its bf16 GELU' map).  Per tensor: relative L2 within 1.3x the
    emulation's own (+ 1e-2 for tensors whose emulated error is tiny) and max error (of the tensor's
    max, a one-element metric) within 1.8x (+ 2e-2).  The two are independent rounding realisations
    of the same storage points, so the GPU is not closer to the emulation than to the exact oracle;
    the claim is the magnitude: the SwinIR tile bounds (l2 / max error ~0.1 on LayerNorm weights,
    test_swinir_m_workload_tile_bf16) are the cost of bf16 maps, not a LayerNorm-backward /
    table-fold defect, and those bounds are set at 1.3x the emulated worst (0.081 L2, 0.136 max)."""
    from basicsr4rs_amd.archs import build_network
    cfg = SWINIR_M2
    torch.manual_seed(0)
    net = build_network(dict(cfg))
    sd = {k: _bf16_round(v.detach()) for k, v in net.state_dict().items()}
    net.load_state_dict(sd)
    x = _bf16_round(torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1)))

    def oracle_grads(emulate):
        sdg = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
        if emulate:
            with O.bf16_storage(grads=True):
                out = O.swinir(sdg, x.double(), cfg)
        else:
            out = O.swinir(sdg, x.double(), cfg)
        g = torch.randn(out.shape, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
        (out * g).sum().backward()
        return {k: v.grad for k, v in sdg.items() if torch.is_tensor(v) and v.grad is not None}, g

    ref, g = oracle_grads(False)
    emu, _ = oracle_grads(True)
    gn = net.to(cuda)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = gn(x.to(cuda))
    (out.float() * g.float().to(cuda)).sum().backward()

    def l2(a, b):
        return (a - b).norm().item() / max(1e-12, b.norm().item())

    def mx(a, b):
        return (a - b).abs().max().item() / max(1e-12, b.abs().max().item())

    rows, bad = [], []
    for n, p in gn.named_parameters():
        a, r, e = p.grad.detach().cpu().double(), ref[n], emu[n]
        row = (n, l2(a, r), l2(e, r), mx(a, r), mx(e, r))
        rows.append(row)
        if row[1] > L2_RATIO * row[2] + 1e-2 or row[3] > MAX_RATIO * row[4] + 2e-2:
            bad.append(row)
    rows.sort(key=lambda r: -r[1])
    for n, gl2, el2, gmx, emx in rows[:6]:
        print(f'{n}: gpu-vs-exact L2 {gl2:.3e} (emulated {el2:.3e}), max {gmx:.3e} (emulated {emx:.3e})')
    r_l2 = max(r[1] / max(r[2], 1e-12) for r in rows)
    r_mx = max(r[3] / max(r[4], 1e-12) for r in rows)
    print(f'worst GPU / emulated ratio over {len(rows)} tensors: L2 {r_l2:.3f}, max {r_mx:.3f}; worst emulated '
          f'L2 {max(r[2] for r in rows):.3e}, max {max(r[4] for r in rows):.3e}')
    assert not bad, bad


# the generic tile conv: since round 6 the W 256 / 512 convs of the HR tails (RRDBNet conv_up1 / conv_up2 /
# conv_hr and their dgrads, the 8-channel conv_last dgrads) run the band kernel over 128-px column strips
GENERIC = ('conv3x3_fwd_kernel<bf16,128,64>', )


def test_rcan_workload_tile_bf16(cuda):
    # B 8: 512 LR rows over 256 band blocks, two rows per band (the bench's B 32 has eight)
    _run(cuda, RCAN, 8, 64, ['conv3x3_fwd_band_kernel', 'conv3x3_wgrad_ring_kernel+reduce', 'conv3x3_fwd_pph_kernel',
                             'conv3x3_fwd_tail_kernel'], out_tol=5e-3, grad_tol=0.12, l2_tol=0.075, absent=GENERIC)


def test_rrdb_workload_tile_bf16(cuda):
    _run(cuda, RRDB, 2, 128, ['conv3x3_fwd_band_kernel', 'conv3x3_fwd_halo_kernel', 'conv3x3_wgrad_ring_kernel+reduce',
                              'conv3x3_fwd_tail_kernel'], out_tol=5e-3, grad_tol=0.15, l2_tol=0.11, absent=GENERIC)


def test_edsr_l_workload_tile_bf16_fwd_bwd(cuda):
    # every 256-channel weight gradient (body and the pixel-shuffled upsample convs) on the kernel-row form
    _run(cuda, EDSR_L4, 2, 64, ['conv3x3_fwd_pph_kernel', 'conv3x3_fwd_tail_kernel', 'conv3x3_wgrad_row3_kernel+reduce'],
         out_tol=5e-3, grad_tol=0.13, l2_tol=0.085, absent=('conv3x3_wgrad_pp_kernel+reduce',))


def test_swinir_m_workload_tile_bf16(cuda):
    # both halves of every block run fused (swin_attn_block_fwd_kernel, swin_mlp_block_fwd_kernel,
    # round 4); the backward keeps its kernels
    _run(cuda, SWINIR_M2, 2, 64, ['swin_attn_block_fwd_kernel', 'swin_mlp_block_fwd_kernel', 'wattn_bwd_kernel',
                                  'linear_wgrad_kernel+reduce', 'linear_wk_kernel', 'conv3x3_wgrad_ring_kernel+reduce'],
         out_tol=5e-3, grad_tol=0.15, l2_tol=0.105)  # <= 1.3x the emulated storage error (test above)


def test_rcan_b32_bench_geometry_bf16(cuda):
    """RCAN at the bench's batch (B 32 x 64^2 LR, C3) with 1 group x 1 RCAB: the band kernels' rows per
    band and the ring wgrad's split plan are those of the benchmarked step (the B 8 tile above runs
    a quarter of them), checked against fp64 instead of only graph == eager."""
    _run(cuda, dict(RCAN, num_group=1, num_block=1), 32, 64,
         ['conv3x3_fwd_band_kernel', 'conv3x3_wgrad_ring_kernel+reduce', 'conv3x3_fwd_pph_kernel',
          'conv3x3_fwd_tail_kernel'], out_tol=5e-3, grad_tol=0.07, l2_tol=0.06, absent=GENERIC)


def test_rrdb_full_depth_error_is_bf16_storage_rounding(cuda):
    """RRDBNet x4 at its full 23 RRDB, 128x128 LR, forward: the HIP bf16 output against the fp32
    oracle (on bf16-rounded weights / input) has the error the oracle itself shows once every stored
    activation is rounded to bf16 (oracle.nets.bf16_storage): within 3 dB of PSNR and 2x of max
    error.  So the bench's RRDB parity (max-abs 0.0255 / 46.1 dB) is the expected cost of bf16
    activations through 345 chained convs, not a kernel defect."""
    from basicsr4rs_amd.archs import build_network
    cfg = dict(RRDB, num_block=23)
    torch.manual_seed(7)
    net = build_network(dict(cfg)).eval()
    sd = {k: _bf16_round(v.detach()) for k, v in net.state_dict().items()}
    net.load_state_dict(sd)
    x = _bf16_round(torch.rand(1, 3, 128, 128, generator=torch.Generator().manual_seed(3)))
    with torch.no_grad():
        ref = O.rrdbnet(sd, x, scale=4, num_block=23)
        with O.bf16_storage():
            emu = O.rrdbnet(sd, x, scale=4, num_block=23)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = net.to(cuda)(x.to(cuda)).float().cpu()

    def stats(a):
        d = a - ref
        return d.abs().max().item(), 10 * math.log10(1.0 / max(1e-30, (d**2).mean().item()))

    (m_gpu, p_gpu), (m_emu, p_emu) = stats(out), stats(emu)
    print(f'RRDBNet x4 23 RRDB bf16: GPU max-abs {m_gpu:.4f} / {p_gpu:.1f} dB; oracle with bf16 storage '
          f'max-abs {m_emu:.4f} / {p_emu:.1f} dB (both against the fp32 oracle)')
    assert p_emu - 3.0 <= p_gpu, (p_gpu, p_emu)
    assert m_gpu <= 2.0 * m_emu + 1e-3, (m_gpu, m_emu)
