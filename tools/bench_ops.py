"""Timing of the basicsr/ops replacements at the SURVEY.md §8 shapes (HIP events).

DCNv2: C5 op config x [16,64,128,128], offset [16,144,128,128], mask [16,72,128,128],
W [64,64,3,3], dg 8 (EDVR PCD, basicsr/archs/edvr_arch.py:42).  upfirdn2d / fused_act:
StyleGAN2 shapes.  Prints per-op ms and algorithmic GB/s (minimum HBM bytes).
"""
import argparse
import json

import torch

from basicsr4rs_amd import _lib
from basicsr4rs_amd.ops import dcn as D
from basicsr4rs_amd.ops.upfirdn2d import upfirdn2d


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--offset-scale', type=float, default=2.0, help='std of the synthetic offsets (pixels)')
    ap.add_argument('--only', default='', help='comma list: dcn,ufd,fba')
    args = ap.parse_args()
    dev = torch.device('cuda')
    res = {}
    N, C, H, W, dg = args.batch, 64, 128, 128, 8
    x = torch.randn(N, C, H, W, device=dev, requires_grad=True)
    off = (torch.randn(N, dg * 18, H, W, device=dev) * args.offset_scale).requires_grad_()
    msk = torch.rand(N, dg * 9, H, W, device=dev, requires_grad=True)
    w = (torch.randn(C, C, 3, 3, device=dev) * 0.05).requires_grad_()
    b = torch.zeros(C, device=dev, requires_grad=True)
    dy = torch.randn(N, C, H, W, device=dev)
    # minimum bytes: read x, offset, mask, write y (fwd); + read dy, write dx, doff, dmask (bwd)
    fwd_bytes = 4 * (x.numel() + off.numel() + msk.numel() + dy.numel())
    only = set(args.only.split(',')) if args.only else {'dcn', 'ufd', 'fba'}
    for mode in (('fp32', 'bf16') if 'dcn' in only else ()):
        ac = mode == 'bf16'

        def fwd():
            with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16, enabled=ac):
                return D.modulated_deform_conv(x, off, msk, w, b, 1, 1, 1, 1, dg)

        def fwdbwd():
            with torch.autocast('cuda', dtype=torch.bfloat16, enabled=ac):
                y = D.modulated_deform_conv(x, off, msk, w, b, 1, 1, 1, 1, dg)
            y.backward(dy)

        tf = timeit(fwd)
        tfb = timeit(fwdbwd, iters=10)
        res[f'dcnv2_{mode}'] = {'fwd_ms': tf, 'fwd_bwd_ms': tfb, 'fwd_alg_GBps': fwd_bytes / tf / 1e6,
                                'fwd_bwd_alg_GBps': 2 * fwd_bytes / tfb / 1e6}
    if 'ufd' not in only:
        print(json.dumps(res, indent=1))
        return
    # upfirdn2d: StyleGAN2 1024 upsample (x2, 4x4 kernel) on [4, 64, 512, 512]
    k = torch.tensor([1., 3., 3., 1.], device=dev)
    k = torch.outer(k, k)
    k = k / k.sum()
    xu = torch.randn(4, 64, 512, 512, device=dev)
    t = timeit(lambda: upfirdn2d(xu, k, up=2, down=1, pad=(2, 1)))
    res['upfirdn2d_up2'] = {'ms': t, 'alg_GBps': 4 * xu.numel() * 5 / t / 1e6}
    t = timeit(lambda: upfirdn2d(xu, k, up=1, down=2, pad=(1, 1)))
    res['upfirdn2d_down2'] = {'ms': t, 'alg_GBps': 4 * xu.numel() * 1.25 / t / 1e6}
    # fused bias act (generic op) on [16, 512, 64, 64]
    xa = torch.randn(16, 512, 64, 64, device=dev)
    ba = torch.randn(512, device=dev)
    out = torch.empty_like(xa)
    lib = _lib.load()

    def fba():
        lib.sr_fused_bias_act(0, _lib.ptr(xa), _lib.ptr(ba), None, _lib.ptr(out), xa.numel(), 64 * 64, 512, 3, 0,
                              0.2, 2**0.5, _lib.stream())

    t = timeit(fba)
    res['fused_bias_act'] = {'ms': t, 'alg_GBps': 8 * xa.numel() / t / 1e6}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
