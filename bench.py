"""North-star benchmark: HR-pixels/sec of the x4 SR train step (BASELINE.json:metric).

Workload (BASELINE.json configs[1]): EDSR_Lx4 (32 ResidualBlockNoBN, nf=256, res_scale=0.1)
train step in bf16, per-GPU batch 32 x 3 x 64 x 64 LR -> 32 x 3 x 256 x 256 HR (HR tile
256 = gt_size).  A step = SRModel.optimize_parameters: forward, L1 loss,
backward, gradient all-reduce (N>1, RCCL), fused Adam(0.9, 0.99) + EMA(0.999).  Inputs
are synthetic U[0,1) tiles already resident in HBM (seed 0 / 1, + rank).

Run: python bench.py --gpus N --steps K --warmup W.  N > 1 runs one rank per GPU (RCCL): under
torch.distributed.run as launched by the driver, or -- started plainly -- bench.py itself starts
torch.distributed.run with N ranks as a child process before touching the GPU.  A WORLD_SIZE from a
launcher that disagrees with --gpus is an error.
A plain N = 1 run (no --workload) is a suite: the EDSR_Lx4 headline (C2) plus one sub-record per
other BASELINE config in the same HR-pixels/s unit (rcan = C3, swinir = C4, rrdb = C5), each
measured in its own child process by `bench.py --workload X` (run_suite; the parent never touches
the GPU).  `--workload X` measures one workload in this process; `--lr-px 256` is the SURVEY §8
secondary sweep (LR 256 -> HR 1024).
Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (HIP events on an
untimed warm-up step; bound chosen from its arithmetic intensity against the 312 FLOP/B
ridge), the CPU baseline (oracle restatement of the same workload's train step on the host
cores, bounded sample, rank 0 at N=1) and the parity of the benchmarked net against the CPU
oracle on one LR tile (fp32 max-abs, bf16 PSNR; rank 0 at N=1, outside the timed region).
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = 'HR-pixels/sec/node (x4 SR train step) + PSNR parity vs CPU ref'
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0

EDSR_L = dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=256, num_block=32, upscale=4, res_scale=0.1,
              img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])


RCAN_X4 = dict(type='RCAN', num_in_ch=3, num_out_ch=3, num_feat=64, num_group=10, num_block=20, squeeze_factor=16,
               upscale=4, res_scale=1, img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])
SWINIR_M = dict(type='SwinIR', upscale=4, in_chans=3, img_size=64, window_size=8, img_range=1.,
                depths=[6, 6, 6, 6, 6, 6], embed_dim=180, num_heads=[6, 6, 6, 6, 6, 6], mlp_ratio=2,
                upsampler='pixelshuffle', resi_connection='1conv')
RRDB_X4 = dict(type='RRDBNet', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=23, num_grow_ch=32, scale=4)

# workload -> (network, model_type, lr, per-GPU batch, LR tile, train FLOPs per HR pixel, label)
# (the FLOPs per HR pixel do not depend on the tile: convs and linears are per pixel, window attention
# per token with a fixed window)
WORKLOADS = {
    'edsr': (EDSR_L, 'SRModel', 1e-4, 32, 64, 18.85e6,
             'EDSR_Lx4 train step (32 RB, nf 256, res_scale 0.1)'),
    'rcan': (RCAN_X4, 'SRModel', 1e-4, 32, 64, 5.97e6,
             'RCAN x4 train step (10 groups x 20 RCAB, nf 64, squeeze 16)'),
    'swinir': (SWINIR_M, 'SwinIRModel', 2e-4, 32, 64, 4.90e6,
               'SwinIR-M x4 classical-SR train step (embed 180, 6x6 STB, 6 heads, window 8)'),
    'rrdb': (RRDB_X4, 'SRModel', 1e-4, 16, 128, 6.72e6,
             'RRDBNet x4 train step (nf 64, gc 32, 23 RRDB)'),
}
# BASELINE.json config each workload line is quoted on
BASELINE_CONFIG = {'edsr': 'configs[1]', 'rcan': 'configs[2]', 'swinir': 'configs[3]', 'rrdb': 'configs[4]'}
# the workloads a plain `python bench.py` (N = 1) reports beside the EDSR headline, one child process each
SUB_WORKLOADS = ('rcan', 'swinir', 'rrdb')


def workload_label(workload, lr_px):
    tile = f'LR {lr_px}x{lr_px} -> HR {4 * lr_px}x{4 * lr_px}'
    if workload == 'rrdb' and lr_px == 128:
        tile += ' (remote-sensing tile)'
    return f'{WORKLOADS[workload][6]}, {tile}'


# train.async_wgrad per workload (weight gradients on a side stream, ops.conv.async_wgrad), from A/B
# runs in one GPU call: RCAN graph 38.9 -> 37.4 ms but eager 54.5 -> 71.5 ms (its eager step is
# host-bound: 2.7k launches, and the fork / record_stream per weight gradient add host time), so
# RCAN takes it only with the HIP graph; SwinIR eager 49.1 -> 46.8 ms; EDSR 40.4 -> 41.4 and RRDB
# 65.6 -> 66.9 ms (two full-chip MFMA kernels interfering), so those stayed single-stream.  Round 4,
# with one fork per block (ops.conv.side_batch): RRDB under the graph 66.9 -> 64.6 ms, so it takes it;
# EDSR still does not (box-dependent: -0.2 ms on one box, +0.6..1.2 ms on another)
ASYNC_WGRAD = {'rcan': 'graph', 'swinir': True, 'rrdb': 'graph'}
# blocks per side-stream fork (ops.conv.side_batch; RCAB / STB / RRDB / ResBlock): one everywhere
# (RCAN 2 / 4 / 20: +0.2 / +0.2 / +1.5 ms; EDSR stays single-stream: with the side stream 37.7 vs
# 37.9 ms on one box, 39.0-39.7 vs 38.4-38.5 on another, profiles/r04/side_batch/)
ASYNC_BLOCKS = {}
for _wl in os.environ.get('SR_BENCH_ASYNC', '').split(','):  # A/B: side-stream weight gradients under the graph
    if _wl:
        ASYNC_WGRAD[_wl] = 'graph'
# bf16 parity floor per workload: PSNR (dB) of the bf16 output against the fp32 CPU oracle on one
# LR tile (parity_check).  Round-2 observations 71.7 / 52.8 / 66.3 / 46.1 dB; the floors sit ~4-6 dB
# below them (RRDB's level is bf16 storage rounding through 345 chained convs:
# tests/test_workload_tiles_gpu.py::test_rrdb_full_depth_error_is_bf16_storage_rounding).  A run
# below its floor exits non-zero after printing its line.
PSNR_FLOOR_BF16 = {'edsr': 66.0, 'rcan': 48.0, 'swinir': 60.0, 'rrdb': 42.0}
# single-process step mode: HIP-graph replay except SwinIR, whose eager step with side-stream weight
# gradients runs 46.7-47.2 ms against 49.0 ms replayed (the replay overlaps the two streams less)
GRAPH_DEFAULT = {'swinir': False}


def make_opt(world, batch, workload='edsr', graph=False, ddp=None, shared_gpu=False):
    net, mtype, lr = WORKLOADS[workload][:3]
    aw = ASYNC_WGRAD.get(workload, False)
    # side-stream weight gradients need a GPU per rank: with several ranks on one GPU (the gloo
    # rehearsal) the segmented DDP graph step with them stalls for seconds once the host runs ahead
    # (RCAN 5.9-13 s / step; with a device sync per segment 97 ms): the ranks' multi-queue graphs
    # with cross-queue waits compete for one GPU's queues (profiles/r04/ddp_async/).
    # The model applies the same guard (models/sr_model.py).
    aw = bool(aw) and not shared_gpu and (graph if aw == 'graph' else True)
    return dict(
        model_type=mtype, is_train=True, dist=world > 1 if ddp is None else ddp, num_gpu=1, rank=0, world_size=world,
        network_g=dict(net),
        train=dict(ema_decay=0.999, use_amp=True, cuda_graph=graph, async_wgrad=aw,
                   async_wgrad_blocks=ASYNC_BLOCKS.get(workload, 1),
                   optim_g=dict(type='Adam', lr=lr, weight_decay=0, betas=[0.9, 0.99]),
                   scheduler=dict(type='MultiStepLR', milestones=[200000], gamma=0.5),
                   pixel_opt=dict(type='L1Loss', loss_weight=1.0, reduction='mean')),
        path={})


def _oracle_fn(net_cfg):
    """CPU oracle forward (oracle/nets.py) of a workload's net: fn(state_dict, x) -> y."""
    from oracle import nets as O
    t = net_cfg['type']
    if t == 'EDSR':
        return lambda sd, x: O.edsr(sd, x, num_block=net_cfg['num_block'], upscale=net_cfg['upscale'],
                                    res_scale=net_cfg['res_scale'], img_range=net_cfg['img_range'],
                                    rgb_mean=net_cfg['rgb_mean'])
    if t == 'RCAN':
        return lambda sd, x: O.rcan(sd, x, num_group=net_cfg['num_group'], num_block=net_cfg['num_block'],
                                    upscale=net_cfg['upscale'], res_scale=net_cfg['res_scale'],
                                    img_range=net_cfg['img_range'], rgb_mean=net_cfg['rgb_mean'])
    if t == 'RRDBNet':
        return lambda sd, x: O.rrdbnet(sd, x, scale=net_cfg['scale'], num_block=net_cfg['num_block'])
    if t == 'SwinIR':
        return lambda sd, x: O.swinir(sd, x, net_cfg)
    raise ValueError(t)


def _cpu_model():
    """The host CPU's model string (/proc/cpuinfo) and its logical CPU count."""
    try:
        with open('/proc/cpuinfo') as f:
            names = [ln.split(':', 1)[1].strip() for ln in f if ln.startswith('model name')]
    except OSError:
        names = []
    return f'{names[0] if names else "unknown"} ({os.cpu_count()} logical CPUs visible)'


def _cpu_threads():
    """Threads for the CPU baseline and why: the host's usable CPUs (affinity mask), capped by the
    CPU share the GPU box grants this job (OMP_NUM_THREADS, which the harness sets to 16 per GPU:
    os.cpu_count() there reports the whole 8-GPU host, and more threads than the share only
    oversubscribe it)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    share = os.environ.get('OMP_NUM_THREADS')
    if share and share.isdigit() and 0 < int(share) < usable:
        return int(share), (f'{share} threads = the CPU share granted per GPU job (OMP_NUM_THREADS); '
                            f'{usable} usable / {os.cpu_count()} logical CPUs on the host')
    return usable, f'all {usable} usable CPUs (affinity mask; {os.cpu_count()} logical)'


def cpu_baseline(workload, seconds=20.0, lr_px=None):
    """The oracle train step of ``workload`` (fwd + L1 + bwd + torch Adam) in torch-CPU fp32 at
    batch 1 on the host's cores: ONE image of the benchmarked tile, timed as the median of as
    many steps as fit in ~``seconds`` (at least 1 after a warm-up).  SwinIR runs eval-mode
    attention (no stochastic depth: its draws only change which samples a branch skips).
    Threads: _cpu_threads (the job's CPU share, stated with the host's width in the line)."""
    from basicsr4rs_amd.archs import build_network
    from oracle import nets as O
    nthr, why = _cpu_threads()
    prev_thr = torch.get_num_threads()
    torch.set_num_threads(nthr)
    net_cfg, _, lr, _, lr_def = WORKLOADS[workload][:5]
    lr_px = lr_px or lr_def
    torch.manual_seed(42)
    net = build_network(dict(net_cfg))
    params = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in net.state_dict().items()}
    opt = torch.optim.Adam([v for v in params.values() if v.requires_grad], lr=lr, betas=(0.9, 0.99))
    g0, g1 = torch.Generator().manual_seed(0), torch.Generator().manual_seed(1)
    lq = torch.rand(1, 3, lr_px, lr_px, generator=g0)
    gt = torch.rand(1, 3, 4 * lr_px, 4 * lr_px, generator=g1)
    fwd = _oracle_fn(net_cfg)

    def step():
        opt.zero_grad()
        O.l1_loss(fwd(params, lq), gt).backward()
        opt.step()

    t = time.time()
    step()  # warm-up
    warm = time.time() - t
    times = []
    t_all = time.time()
    while not times or (time.time() - t_all + warm < seconds and len(times) < 10):
        t = time.time()
        step()
        times.append(time.time() - t)
    times.sort()
    t_med = times[len(times) // 2]
    torch.set_num_threads(prev_thr)
    return {'value': (4 * lr_px)**2 / t_med, 'unit': 'HR-pixels/s', 'cores': nthr, 'kind': 'port',
            'cpu_model': _cpu_model(), 'cores_note': why,
            'sample': f'oracle {net_cfg["type"]} fp32 train step (fwd + L1 + bwd + Adam), batch 1 '
                      f'({lr_px}x{lr_px} LR -> {4 * lr_px}x{4 * lr_px} HR), median of {len(times)} steps after '
                      f'1 warm-up, torch CPU threads={nthr}'}


def parity_check(workload, dev):
    """Parity of the benchmarked net against the CPU oracle on ONE LR tile of the bench size
    (outside the timed region; same random-init weights and input): fp32 max |GPU - CPU| (the
    north_star bar is 1e-3) and the PSNR of the bf16 (autocast) GPU output against the fp32 CPU
    output, with the [0,1] image range as peak."""
    import copy

    from basicsr4rs_amd.archs import build_network
    net_cfg, lr_px = WORKLOADS[workload][0], WORKLOADS[workload][4]
    torch.manual_seed(7)
    net = build_network(dict(net_cfg)).eval()
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    x = torch.rand(1, 3, lr_px, lr_px, generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = _oracle_fn(net_cfg)(sd, x)
        g = copy.deepcopy(net).to(dev)
        out32 = g(x.to(dev)).float().cpu()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out16 = g(x.to(dev)).float().cpu()

    def psnr(a):
        mse = ((a - ref)**2).mean().item()
        return round(10 * math.log10(1.0 / mse), 2) if mse > 0 else float('inf')

    return {'max_abs_fp32': float((out32 - ref).abs().max()), 'psnr_fp32_db': psnr(out32),
            'max_abs_bf16': float((out16 - ref).abs().max()), 'psnr_bf16_db': psnr(out16),
            'tile': f'1x3x{lr_px}x{lr_px} LR, eval mode, oracle = oracle/nets.py CPU fp32',
            'bar': f'fp32 max-abs <= 1e-3 (north_star); bf16 PSNR >= {PSNR_FLOOR_BF16[workload]} dB'}


def swin_fused_roofline(model, batch, lr_px, dev, reps=20):
    """North-star check 'MFMA peak on SwinIR window attention': the fused attention half of one
    SwinTransformerBlock (LN1 -> qkv -> shifted-window attention -> proj + residual,
    swin_attn_block_fwd_kernel) timed on its own with HIP events on the bench's token map
    (B x 64 x 64 x 184 bf16), training mode (ln1 / qkv / attention output / lse written for the
    backward) and inference mode (x2 only), plus the fused MLP half.  FLOPs are algorithmic
    (qkv + QK^T + AV + proj, unpadded); fraction of the 2.5 PF dense bf16 peak."""
    from basicsr4rs_amd.ops import swin as S
    net = model.get_bare_model(model.net_g)
    blk = net._blocks()[1]  # a shifted block
    at = blk.attn
    g, fc1s, fc2s = blk._geom, blk._fc1, blk._fc2
    Cp = fc1s.cin_p
    x = torch.randn(batch, lr_px, lr_px, Cp, device=dev).to(torch.bfloat16)
    x[..., g.dim:] = 0
    qwf, _, qbg = S.prepared_linear(at.qkv.weight, at.qkv.bias, g.qkv, torch.bfloat16)
    pwf, _, pbg = S.prepared_linear(at.proj.weight, at.proj.bias, g.proj, torch.bfloat16)
    f1wf, _, f1bg = S.prepared_linear(blk.mlp.fc1.weight, blk.mlp.fc1.bias, fc1s, torch.bfloat16)
    f2wf, _, f2bg = S.prepared_linear(blk.mlp.fc2.weight, blk.mlp.fc2.bias, fc2s, torch.bfloat16)
    tab = at.relative_position_bias_table.detach().float().contiguous()
    out = {}
    calls = {
        'attention_train': lambda: S.swin_attn_fused(x, blk.norm1.weight, blk.norm1.bias, g.dim, qwf, qbg, tab, pwf, pbg,
                                                     None, g, float(at.scale), True),
        'attention_inference': lambda: S.swin_attn_fused(x, blk.norm1.weight, blk.norm1.bias, g.dim, qwf, qbg, tab, pwf,
                                                         pbg, None, g, float(at.scale), False),
        'mlp_train': lambda: S.swin_mlp_fused(x, blk.norm2.weight, blk.norm2.bias, g.dim, f1wf, f1bg, fc1s, f2wf, f2bg,
                                              None, True),
    }
    N, H, W = batch, lr_px, lr_px
    flops = {'attention_train': S.attn_block_flops(g, N, H, W), 'attention_inference': S.attn_block_flops(g, N, H, W),
             'mlp_train': 4.0 * N * H * W * fc1s.cin * fc1s.cout}
    with torch.no_grad():
        for name, fn in calls.items():
            if fn() is None:
                return None
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / reps * 1e3
            tf = flops[name] / (us * 1e-6) / 1e12
            out[name] = {'us': round(us, 2), 'tflops': round(tf, 1), 'frac_mfma_peak': round(tf / PEAK_BF16_TFLOPS, 4)}
    out['kernels'] = 'swin_attn_block_fwd_kernel / swin_mlp_block_fwd_kernel'
    out['flops'] = 'attention: qkv + QK^T + AV + proj (unpadded C 180, head dim 30); mlp: fc1 + fc2'
    return out


def _pmc_traffic(workload, kernel):
    """HBM bytes per launch of ``kernel`` from this round's committed PMC passes
    (tools/profile_round.sh -> profiles/pmc_traffic.json), or None."""
    try:
        recs = json.load(open(os.path.join(ROOT, 'profiles', 'pmc_traffic.json')))
    except (OSError, ValueError):
        return None
    # the workload's record, or one of its extra kernels' (key '<workload>_<what>'): the dominant
    # kernel of a step can change between close contenders (SwinIR linear_wk / linear_wgrad)
    for key, rec in sorted(recs.items()):
        if (key == workload or key.startswith(workload + '_')) and rec.get('bench_kernel') == kernel and \
                rec.get('hbm_bytes_per_launch') is not None:
            return rec
    return None


def _roof(flops, nbytes, sec):
    """(bound, achieved, peak, unit, frac) of one launch: bound from its algorithmic arithmetic
    intensity against the ridge (frac = achieved / min(P, AI * BW))."""
    ai = flops / nbytes if nbytes > 0 else float('inf')
    ridge = PEAK_BF16_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)
    if flops > 0 and ai >= ridge:
        a = flops / sec / 1e12
        return 'mfma', a, PEAK_BF16_TFLOPS, 'TFLOP/s', a / PEAK_BF16_TFLOPS
    a = nbytes / sec / 1e9
    return 'hbm', a, PEAK_HBM_GBS, 'GB/s', a / PEAK_HBM_GBS


def roofline(workload, kstats, traced_steps, step_s, use_graph):
    """Roofline of the dominant kernel (most time in the traced step), per KERNEL LAUNCH:
    flops / bytes per launch = the traced calls' algorithmic totals / their launches (a sliced band
    call is several launches; a wgrad span is its kernel + slab reduce, one 'launch' pair).  Three
    durations per launch: in-step HIP events around every launch of the traced eager step (launches
    back to back behind a spin kernel; the headline ``frac``), the same launches re-issued back to
    back in isolation after the timed region (``frac_isolated``), and the rocprofv3 average inside
    the timed graph replays from this round's committed --stats summary (``frac_rocprof``)."""
    name, st = max(kstats.items(), key=lambda kv: kv[1]['ms'])
    calls, launches = st['count'], st['launches']
    lpc = launches / calls
    step_ms = st['ms'] / traced_steps
    in_step_s = st['ms'] * 1e-3 / launches
    fl, by = st['flops'] / launches, st['bytes'] / launches
    bound, ach, peak, unit, frac = _roof(fl, by, in_step_s)
    roof = {'bound': bound, 'kernel': name, 'achieved': round(ach, 1), 'peak': peak, 'unit': unit,
            'frac': round(frac, 4), 'traffic': None, 'flops_per_launch': fl, 'bytes_per_launch': by,
            'arith_intensity': round(fl / by, 1) if by else None, 'ridge': round(PEAK_BF16_TFLOPS / PEAK_HBM_GBS * 1e3, 1),
            'launches_per_step': launches // traced_steps, 'calls_per_step': calls // traced_steps,
            'avg_launch_us': round(in_step_s * 1e6, 2), 'share_of_step': round(step_ms * 1e-3 / step_s, 3)}
    if bound == 'hbm' and fl > 0:
        roof['mfma_tflops'] = round(fl / in_step_s / 1e12, 1)
    from basicsr4rs_amd.utils import ktrace
    rel_ms = ktrace.time_relaunch(name)  # per call
    ktrace.clear_relaunch()
    if rel_ms is not None:
        iso_s = rel_ms * 1e-3 / lpc
        roof['avg_launch_us_isolated'] = round(iso_s * 1e6, 2)
        roof['frac_isolated'] = round(_roof(fl, by, iso_s)[4], 4)
    tr = _pmc_traffic(workload, name)
    if tr:
        if tr.get('hbm_bytes_per_launch') is not None:
            roof['traffic'] = round(tr['hbm_bytes_per_launch'])
        if tr.get('rocprof_avg_us'):
            roof['rocprof_avg_us'] = round(tr['rocprof_avg_us'], 2)
            roof['frac_rocprof'] = round(_roof(fl, by, tr['rocprof_avg_us'] * 1e-6)[4], 4)
        roof['traffic_source'] = (f"{tr['source']}: rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE (own passes) per launch of "
                                  f"{tr['kernel_regex']}, {tr['correction']}; rocprof_avg_us: --kernel-trace --stats "
                                  f"average per launch in the timed graph replays ({tr.get('stats_file', '')})")
    roof['timing'] = ('avg_launch_us: HIP events around each launch of the traced ' +
                      ('eager step before capture (replays run the same kernels)' if use_graph else
                       'last (untimed) warm-up step') + ', single stream, launches back to back behind a spin kernel; '
                      'avg_launch_us_isolated: the same launches re-issued back to back after the timed region '
                      '(3 passes after a warm-up pass)')
    roof['kernels'] = {
        k: {'calls': v['count'] // traced_steps, 'launches': v['launches'] // traced_steps,
            'avg_us': round(v['ms'] / v['launches'] * 1e3, 1),
            'tflops': round(v['flops'] / (v['ms'] * 1e-3) / 1e12, 1) if v['ms'] > 0 and v['flops'] else None,
            'gbs': round(v['bytes'] / (v['ms'] * 1e-3) / 1e9, 1) if v['ms'] > 0 else None,
            'ms_per_step': round(v['ms'] / traced_steps, 3)}
        for k, v in sorted(kstats.items(), key=lambda kv: -kv[1]['ms'])
    }
    return roof


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """``--gpus N`` (N > 1) started as a plain ``python bench.py``: run the N rank processes (one
    per GPU, RCCL) under torch.distributed.run as a CHILD process -- this process has not touched
    the GPU and never does -- and return its exit code (rank 0 prints the one JSON line)."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', f'--master-port={_free_port()}', os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')  # dmabuf IPC only on this host driver
    return subprocess.call(cmd, env=env)


def _config(workload, B, world, use_graph, async_wgrad, lr_px):
    wl = WORKLOADS[workload]
    return {'workload': workload_label(workload, lr_px), 'baseline_config': BASELINE_CONFIG[workload],
            'global_batch': B * world, 'per_gpu_batch': B, 'lr_tile': lr_px, 'seq_len': None,
            'parallelism': f'dp{world}', 'model': wl[0]['type'], 'hip_graph': use_graph,
            'async_wgrad': bool(async_wgrad)}


def dry_run(args, world, rank):
    """The launch and reporting skeleton of ``main`` without a GPU: gloo rendezvous, barrier,
    ``--steps`` no-op steps timed between barriers, MAX over ranks, one JSON line from rank 0 with
    the configuration the real run would report (value null: nothing is measured)."""
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group('gloo')
    B = args.batch or WORKLOADS[args.workload][3]
    use_graph = (GRAPH_DEFAULT.get(args.workload, True) or world > 1) if args.graph < 0 else bool(args.graph)
    opt = make_opt(world, B, args.workload, use_graph)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({'metric': BASELINE_METRIC, 'value': None, 'unit': 'HR-pixels/s', 'n_gpus': world,
                          'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': None, 'dry_run': True,
                          'ranks_seen': world, 'max_rank_s': t.item(),
                          'config': _config(args.workload, B, world, use_graph, opt['train']['async_wgrad'],
                                            args.lr_px or WORKLOADS[args.workload][4]),
                          'roofline': None, 'cpu_baseline': None, 'parity': None}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _compact(line):
    """The per-workload summary a suite line carries (kept short: the driver's record keeps the
    last 2000 characters of stdout, so the four summaries sit at the end of the one line)."""
    if line is None:
        return None
    roof, cpu, par, sw = line.get('roofline'), line.get('cpu_baseline'), line.get('parity'), \
        line.get('swin_fused_attention')
    out = {'config': (line.get('config') or {}).get('baseline_config'), 'B': (line.get('config') or {}).get('per_gpu_batch'),
           'lr': (line.get('config') or {}).get('lr_tile'), 'ms_per_step': line.get('ms_per_step'),
           'value': line.get('value'), 'model_tflops': line.get('model_tflops')}
    if roof:
        out['roofline'] = {k: roof.get(k) for k in ('kernel', 'bound', 'achieved', 'peak', 'unit', 'frac', 'traffic')}
    else:
        out['roofline'] = None
    out['cpu_baseline'] = {k: cpu.get(k) for k in ('value', 'cores', 'kind')} if cpu else None
    out['parity'] = {'max_abs_fp32': par.get('max_abs_fp32'), 'psnr_bf16_db': par.get('psnr_bf16_db')} if par else None
    if sw:
        out['swin_attn_frac'] = {k: sw[k]['frac_mfma_peak'] for k in ('attention_train', 'attention_inference', 'mlp_train')
                                 if k in sw}
    return out


def run_suite(args):
    """A plain ``python bench.py`` at N = 1: the EDSR headline and one sub-record per other BASELINE
    workload (SUB_WORKLOADS), each measured by ``bench.py --workload X`` in a CHILD process with the
    same --steps / --warmup.  This process never touches the GPU (it only starts the children, one
    after another, and merges their JSON lines), so every child starts on an idle, freshly
    initialised device.  The printed line is the headline child's line unchanged (value, timing,
    roofline, cpu_baseline of EDSR_Lx4 B 32), plus ``workloads``: a compact summary of all four
    (ms/step, HR-px/s, the dominant kernel's roofline, cpu_baseline, parity; SwinIR's fused-attention
    MFMA fractions) and ``sub_records``: each child's full line.  Exit status: the headline child's;
    a failed sub-workload is recorded in its entry (``rc``) and on stderr."""
    import subprocess
    base = [sys.executable, os.path.abspath(__file__), '--gpus', '1', '--steps', str(args.steps),
            '--warmup', str(args.warmup), '--graph', str(args.graph)]
    for flag in ('no_cpu_baseline', 'no_trace', 'no_parity', 'ddp', 'dry_run'):
        if getattr(args, flag):
            base.append('--' + flag.replace('_', '-'))
    if args.batch:
        base += ['--batch', str(args.batch)]
    if args.lr_px:
        base += ['--lr-px', str(args.lr_px)]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    lines, rcs, walls = {}, {}, {}
    for wl in ('edsr',) + tuple(w for w in args.sub_workloads.split(',') if w):
        cmd = base + ['--workload', wl, '--cpu-seconds', str(args.cpu_seconds if wl == 'edsr' else args.sub_cpu_seconds)]
        t0 = time.time()
        try:
            p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True, timeout=args.child_timeout)
            rc, out = p.returncode, p.stdout
        except subprocess.TimeoutExpired as e:
            rc, out = 124, (e.stdout.decode() if isinstance(e.stdout, bytes) else (e.stdout or ''))
        walls[wl] = round(time.time() - t0, 1)
        js = [ln for ln in out.splitlines() if ln.startswith('{')]
        for ln in out.splitlines():  # the child's other stdout (none expected) stays visible
            if not ln.startswith('{'):
                print(ln, file=sys.stderr)
        lines[wl] = json.loads(js[-1]) if js else None
        rcs[wl] = rc
        if rc != 0:
            print(f'bench: workload {wl} exited {rc}', file=sys.stderr)
        print(f'bench: {wl} done in {walls[wl]} s (rc {rc})', file=sys.stderr, flush=True)
        if wl == 'edsr' and lines[wl] is None:
            return rc or 1
    line = dict(lines['edsr'])
    line['suite'] = {'parent_touches_gpu': False, 'child_wall_s': walls,
                     'note': 'each workload measured by `bench.py --workload X` in its own child process'}
    line['sub_records'] = {wl: lines[wl] for wl in lines if wl != 'edsr'}
    line['workloads'] = {}
    for wl in lines:
        c = _compact(lines[wl]) or {'error': 'no JSON line'}
        c['rc'] = rcs[wl]
        line['workloads'][wl] = c
    print(json.dumps(line), flush=True)
    return rcs['edsr']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (0: the workload default)')
    ap.add_argument('--workload', default=None, choices=sorted(WORKLOADS),
                    help='measure one workload in this process (default: the EDSR headline, plus the '
                         '--sub-workloads as sub-records at N = 1, each in a child process)')
    ap.add_argument('--sub-workloads', default=','.join(SUB_WORKLOADS),
                    help='comma list reported beside the headline when --workload is not given at N = 1 ("" none)')
    ap.add_argument('--lr-px', type=int, default=0,
                    help='LR tile side (0: the workload default, 64; RRDB 128); HR = 4x (SURVEY §8 sweep: 256)')
    ap.add_argument('--cpu-seconds', type=float, default=20.0, help='CPU-baseline sample budget (s)')
    ap.add_argument('--sub-cpu-seconds', type=float, default=12.0, help='the same for each sub-workload (s)')
    ap.add_argument('--child-timeout', type=float, default=900.0, help='per-workload child time limit (s)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-trace', action='store_true')
    ap.add_argument('--no-parity', action='store_true')
    ap.add_argument('--graph', type=int, default=-1,
                    help='capture the train step in a HIP graph (1/0; default: on for a single process)')
    ap.add_argument('--ddp', action='store_true',
                    help='run the distributed step (bucketed reducer, segmented graph, RCCL) also at N=1')
    ap.add_argument('--dry-run', action='store_true',
                    help='launch / rendezvous / barrier / max-over-ranks timing / JSON line only, with a no-op step '
                         'on the CPU (gloo); no GPU, no measurement (tests/test_bench_launch.py)')
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error('--gpus must be >= 1')

    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and args.gpus > 1:
        # `python bench.py --gpus N`: one rank per GPU, launched before anything touches the GPU
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or '1')
    if world != args.gpus:
        print(f'bench: --gpus {args.gpus} disagrees with WORLD_SIZE={world} from the launcher', file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.workload is None:
        if env_world is None and args.sub_workloads:
            sys.exit(run_suite(args))  # N = 1, plain start: headline + sub-records in child processes
        args.workload = 'edsr'
    if args.dry_run:
        return dry_run(args, world, rank)
    ddp = world > 1 or args.ddp
    shared_gpu = world > max(1, torch.cuda.device_count())  # ranks sharing a GPU (gloo rehearsal)
    if ddp:
        from basicsr4rs_amd.utils.dist_util import init_dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if world == 1:  # --ddp on one process: a world of one
            os.environ.setdefault('MASTER_PORT', str(_free_port()))
            os.environ.setdefault('RANK', '0')
            os.environ.setdefault('WORLD_SIZE', '1')
        # RCCL ('nccl') for the real runs; SR_DIST_BACKEND=gloo rehearses the N > 1 path of this
        # script (barriers, max-over-ranks timing, bucketed reducer) with several ranks on one GPU
        init_dist('pytorch', backend=os.environ.get('SR_DIST_BACKEND', 'nccl'))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    from basicsr4rs_amd.utils import ktrace

    torch.manual_seed(42)
    wl = WORKLOADS[args.workload]
    B = args.batch or wl[3]
    lr_px = args.lr_px or wl[4]
    hr_px_tile = (4 * lr_px) ** 2
    # the step as HIP-graph replay (one graph; under DDP a chain of graphs cut at the gradient
    # buckets, utils/step_graph.py), except single-process SwinIR whose eager step is faster
    use_graph = (GRAPH_DEFAULT.get(args.workload, True) or ddp) if args.graph < 0 else bool(args.graph)
    opt = make_opt(world, B, args.workload, use_graph, ddp=ddp, shared_gpu=shared_gpu)
    opt['rank'] = rank
    model = build_model(opt)
    g0 = torch.Generator(device=dev).manual_seed(0 + rank)
    g1 = torch.Generator(device=dev).manual_seed(1 + rank)
    lq = torch.rand(B, 3, lr_px, lr_px, generator=g0, device=dev)
    gt = torch.rand(B, 3, 4 * lr_px, 4 * lr_px, generator=g1, device=dev)
    model.feed_data({'lq': lq, 'gt': gt})

    # The per-kernel HIP-event trace is taken on one untimed warm-up step, never inside the timed
    # region (per-launch events would slow the timed steps).  With a captured step it is the last
    # eager warm-up step (a graph replay runs the same kernels but cannot be instrumented per
    # launch; capture happens on warm-up step 3, so at least 3 warm-up steps run); eager (DDP)
    # runs trace their last warm-up step.
    it = 0
    warmup = max(args.warmup, 3) if use_graph else max(args.warmup, 0 if args.no_trace else 2)
    trace_w = 1 if use_graph else warmup - 1
    kstats, traced_steps = {}, 0
    for w in range(warmup):
        it += 1
        model.update_learning_rate(it)
        if w == trace_w - 1 and not args.no_trace:
            # a spin kernel ahead of the step BEFORE the traced one lets the host run ahead of
            # the GPU, so the traced step's launches run back to back and each event pair
            # brackets its kernel alone (without it, host-issue gaps between short eager kernels
            # -- RCAN: 2.7k launches -- land inside the spans: 45 us vs rocprof's 27 us); the
            # untraced step in between brings the clocks back up after the idle spin
            torch.cuda.synchronize()
            torch.cuda._sleep(int(os.environ.get('SR_TRACE_SLEEP_CYCLES', 400_000_000)))
            model.optimize_parameters(it)
        elif w == trace_w and not args.no_trace:
            ktrace.start()
            model.optimize_parameters(it)
            kstats, traced_steps = ktrace.stop(), 1
        else:
            model.optimize_parameters(it)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        it += 1
        model.update_learning_rate(it)
        model.optimize_parameters(it)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    loss = model.get_current_log().get('l_pix', float('nan'))
    if os.environ.get('SR_STEP_TRACE') and getattr(model, '_graph', None) is not None and \
            hasattr(model._graph, 'trace'):  # segmented DDP replay: per-phase host times (ms) of the last steps
        for tr in model._graph.trace[-3:]:
            ph = [(k, round((t - p) * 1e3, 3)) for (k, t), (_, p) in zip(tr[1:], tr[:-1])]
            print(json.dumps({'rank': rank, 'step_trace': os.environ['SR_STEP_TRACE'], 'phases_ms': ph,
                              'total_ms': round((tr[-1][1] - tr[0][1]) * 1e3, 3)}), file=sys.stderr)

    hr_px = world * B * hr_px_tile * args.steps
    value = hr_px / dt
    roof = None
    if kstats:
        roof = roofline(args.workload, kstats, traced_steps, dt / args.steps, use_graph)
    cpu = parity = swin_att = None
    if rank == 0 and args.workload == 'swinir':
        swin_att = swin_fused_roofline(model, B, lr_px, dev)
    if rank == 0 and world == 1 and not args.no_parity:
        parity = parity_check(args.workload, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.workload, args.cpu_seconds, lr_px)
    if rank == 0:
        line = {
            'metric': BASELINE_METRIC, 'value': round(value, 1), 'unit': 'HR-pixels/s',
            'n_gpus': world, 'steps': args.steps, 'warmup': warmup, 'ms_per_step': round(dt / args.steps * 1e3, 3),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'bf16',
            'data': 'synthetic U[0,1) LR/GT tiles resident in HBM, random-init weights',
            'config': _config(args.workload, B, world, use_graph, opt['train']['async_wgrad'], lr_px),
            'train_flops_per_hr_px': wl[5], 'model_tflops': round(wl[5] * value / 1e12, 1),
            'last_loss': loss, 'cuda_graph': use_graph, 'roofline': roof, 'cpu_baseline': cpu, 'parity': parity,
            'swin_fused_attention': swin_att,
        }
        print(json.dumps(line))
        if not math.isfinite(loss):  # a step that trains on NaNs is not a measurement
            print(f'bench: non-finite training loss {loss}', file=sys.stderr)
            sys.exit(1)
        if parity is not None and (parity['max_abs_fp32'] > 1e-3 or
                                   parity['psnr_bf16_db'] < PSNR_FLOOR_BF16[args.workload]):
            print(f'bench: parity below the bar: {parity}', file=sys.stderr)
            sys.exit(1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
