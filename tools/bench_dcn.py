"""DCNv2 at the C5 op config (BASELINE.json configs[4]):
x [16,64,128,128], offset [16,144,128,128] ~ N(0,1), mask [16,72,128,128] = sigmoid(N(0,1)),
W [64,64,3,3], bias [64], stride 1, pad 1, dilation 1, groups 1, deformable groups 8 (EDVR PCD,
basicsr/archs/edvr_arch.py:42) -- the reference's modulated_deform_conv path
(basicsr/ops/dcn/deform_conv.py:121-188 -> deform_conv_cuda.cpp:490-685).

Times forward and forward + backward in fp32 and bf16 (autocast) with HIP events, reports
algorithmic FLOPs / bytes -- one definition for every DCN number (round 4): each tensor touched once
as the kernels store it: x, dy at the compute dtype (bf16 NHWC under autocast), offset, mask, y and
their gradients and dx in fp32 (the forward: 327 MB at the C5 config in bf16; the backward reads dy,
x, offset, mask and writes dx, doffset, dmask: 587 MB) -- and the roofline fraction
against min(2.5 PF, AI x 8 TB/s) (bf16) / min(157 TF, AI x 8 TB/s) (fp32), and times the CPU
oracle (oracle/ops.py, numpy float64, the restatement of the reference's kernels) on a bounded
sample (batch 1 of the same per-image shape) on the host cores.

Usage (GPU box): python tools/bench_dcn.py [--out profiles/r03/dcn_bench.json] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from basicsr4rs_amd.ops import dcn as D  # noqa: E402

PEAK = {'bf16': 2500e12, 'fp32': 157.3e12}
HBM = 8000e9


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def inputs(N, dev, seed=0):
    g = torch.Generator(device='cpu').manual_seed(seed)
    C, H, W, dg = 64, 128, 128, 8
    x = torch.randn(N, C, H, W, generator=g)
    off = torch.randn(N, dg * 18, H, W, generator=g)
    msk = torch.sigmoid(torch.randn(N, dg * 9, H, W, generator=g))
    w = torch.randn(C, C, 3, 3, generator=g) * 0.05
    b = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(N, C, H, W, generator=g)
    return [t.to(dev) for t in (x, off, msk, w, b, dy)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--out', default='')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--modes', default='fp32,bf16')
    args = ap.parse_args()
    dev = torch.device('cuda')
    N, C, H, W, dg = args.batch, 64, 128, 128, 8
    x, off, msk, w, b, dy = inputs(N, dev)
    for t in (x, off, msk, w, b):
        t.requires_grad_(True)
    P = N * H * W
    flops_fwd = 2.0 * P * C * C * 9
    flops_bwd = 2 * flops_fwd  # dcols = W^T dy and dW = dy cols^T (the coordinate / scatter math not counted)
    res = {'config': 'x[16,64,128,128] offset[16,144,128,128] mask[16,72,128,128] W[64,64,3,3] dg 8, s1 p1 d1 g1',
           'batch': N}
    for mode in args.modes.split(','):
        ac = mode == 'bf16'
        esz = 2 if ac else 4
        om = 4 * (off.numel() + msk.numel())  # offset + mask (or their gradients), fp32
        bytes_fwd = esz * x.numel() + om + 4 * dy.numel()  # x, offset, mask in; y (fp32) out
        bytes_bwd = esz * (dy.numel() + x.numel()) + 2 * om + 4 * x.numel()  # dy, x, off, mask in; dx, doff, dmask out

        def fwd():
            with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, enabled=ac):
                return D.modulated_deform_conv(x, off, msk, w, b, 1, 1, 1, 1, dg)

        def fwdbwd():
            for t in (x, off, msk, w, b):  # as zero_grad(set_to_none=True): no accumulation kernels timed
                t.grad = None
            with torch.autocast('cuda', dtype=torch.bfloat16, enabled=ac):
                y = D.modulated_deform_conv(x, off, msk, w, b, 1, 1, 1, 1, dg)
            y.backward(dy)

        tf = timeit(fwd, args.iters) * 1e-3
        tfb = timeit(fwdbwd, max(5, args.iters // 2)) * 1e-3
        ai_f = flops_fwd / bytes_fwd
        ai_fb = (flops_fwd + flops_bwd) / (bytes_fwd + bytes_bwd)
        roof_f = min(PEAK[mode], ai_f * HBM)
        roof_fb = min(PEAK[mode], ai_fb * HBM)
        res[mode] = {
            'fwd_ms': round(tf * 1e3, 3), 'fwd_bwd_ms': round(tfb * 1e3, 3),
            'fwd_alg_bytes': bytes_fwd, 'fwd_alg_flops': flops_fwd, 'fwd_ai': round(ai_f, 1),
            'fwd_tflops': round(flops_fwd / tf / 1e12, 2), 'fwd_alg_GBps': round(bytes_fwd / tf / 1e9, 1),
            'fwd_roof_tflops': round(roof_f / 1e12, 1), 'fwd_frac': round(flops_fwd / tf / roof_f, 4),
            'fwd_bwd_alg_bytes': bytes_fwd + bytes_bwd, 'fwd_bwd_alg_flops': flops_fwd + flops_bwd,
            'fwd_bwd_ai': round(ai_fb, 1), 'fwd_bwd_tflops': round((flops_fwd + flops_bwd) / tfb / 1e12, 2),
            'fwd_bwd_roof_tflops': round(roof_fb / 1e12, 1),
            'fwd_bwd_frac': round((flops_fwd + flops_bwd) / tfb / roof_fb, 4),
            'bound': 'hbm' if min(ai_f, ai_fb) * HBM < PEAK[mode] else 'mfma',
        }
        print(mode, json.dumps(res[mode]), flush=True)
    if not args.no_cpu:
        from oracle import ops as OO
        xs, offs, msks, ws, bs, dys = [t.numpy() for t in inputs(1, 'cpu', seed=1)]
        t0 = time.time()
        OO.dcn_forward(xs, offs, msks, ws, bs, 1, 1, 1, 1, dg)
        t1 = time.time()
        OO.dcn_backward(xs, offs, msks, ws, bs, 1, 1, 1, 1, dg, dys)
        t2 = time.time()
        res['cpu_baseline'] = {
            'kind': 'port', 'sample': 'batch 1 of the same per-image shape (x[1,64,128,128], dg 8), oracle/ops.py '
                                      'numpy float64 dcn_forward / dcn_backward, one run each',
            'fwd_s_per_image': round(t1 - t0, 3), 'bwd_s_per_image': round(t2 - t1, 3),
            'fwd_img_per_s': round(1 / (t1 - t0), 3), 'fwd_bwd_img_per_s': round(1 / (t2 - t0), 3),
            'cores': 1, 'threads_note': f'numpy ({np.__version__}) einsum / add.at: effectively one core',
            'gpu_fwd_img_per_s_bf16': round(N / (res['bf16']['fwd_ms'] * 1e-3), 1),
            'gpu_fwd_bwd_img_per_s_bf16': round(N / (res['bf16']['fwd_bwd_ms'] * 1e-3), 1)}
        print('cpu', json.dumps(res['cpu_baseline']), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        json.dump(res, open(args.out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
