"""Micro-benchmark of the HIP conv kernels at the EDSR-L shapes (fwd / dgrad / wgrad),
timed with HIP events on the current stream; prints TFLOP/s per kernel."""
import json
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd.ops import conv as C  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = 'cuda'
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else '0').split(',')]
    lib = C._lib.load()
    res = []
    for dtype, variant in [(torch.bfloat16, v) for v in variants]:
        C._lib.check(lib.sr_conv3x3_set_variant(variant))
        shapes = [(256, 256, 64, 0), (256, 1024, 64, 2), (256, 1024, 128, 2), (256, 3, 256, 0), (64, 64, 64, 0)]
        if len(sys.argv) > 3:  # e.g. 256,256,64,0 (cin, cout, hw, out_ps[, ksize]); ';'-separated list
            shapes = [tuple(int(v) for v in sh.split(',')) for sh in sys.argv[3].split(';')]
        for shp in shapes:
            cin, cout, hw, ps = shp[:4]
            ks = shp[4] if len(shp) > 4 else 3
            if ks == 1:  # 1x1 conv = nn.Linear over tokens: fwd and dgrad only
                taps = 1
                x = torch.randn(B, hw, hw, C.pad8(cin), device=dev).to(dtype)
                wf = (torch.randn(C.pad8(cout), C.pad8(cin), device=dev) * 0.05).to(dtype)
                wd = (torch.randn(C.pad8(cin), C.pad8(cout), device=dev) * 0.05).to(dtype)
                y = torch.empty(B, hw, hw, C.pad8(cout), device=dev, dtype=dtype)
                dx = torch.empty(B, hw, hw, C.pad8(cin), device=dev, dtype=dtype)
                fl = 2.0 * B * hw * hw * cin * cout
                t = timeit(lambda: C.conv_fwd_raw(x, wf, None, y, B, hw, hw, C.pad8(cin), C.pad8(cout), cout, ksize=1))
                nb = 2.0 * B * hw * hw * (C.pad8(cin) + C.pad8(cout))  # read X once, write Y once (bf16)
                res.append(dict(v=variant, k='fwd1x1', cin=cin, cout=cout, hw=hw, ms=t, tflops=fl / t / 1e9,
                                gbps=nb / t / 1e6))
                t = timeit(lambda: C.conv_fwd_raw(y, wd, None, dx, B, hw, hw, C.pad8(cout), C.pad8(cin), cin, ksize=1))
                res.append(dict(v=variant, k='dgrad1x1', cin=cin, cout=cout, hw=hw, ms=t, tflops=fl / t / 1e9,
                                gbps=nb / t / 1e6))
                t = timeit(lambda: C.conv_wgrad_raw(y, x, B, hw, hw, C.pad8(cin), cin, C.pad8(cout), cout, ksize=1))
                res.append(dict(v=variant, k='wgrad1x1', cin=cin, cout=cout, hw=hw, ms=t, tflops=fl / t / 1e9,
                                gbps=nb / t / 1e6))  # operand bytes (dy + x once), slab traffic not counted
                continue
            conv = torch.nn.Conv2d(cin, cout, 3, 1, 1).to(dev)
            spec = C.ConvSpec(cin, cout, out_ps=ps, out_nchw=(cout == 3))
            x = torch.randn(B, hw, hw, C.pad8(cin), device=dev).to(dtype)
            wf, wd, bg = C.prepared(conv.weight, conv.bias, spec, dtype)
            shp = C._out_shape(spec, B, hw, hw)
            y = torch.empty(shp, device=dev, dtype=torch.float32 if spec.out_nchw else dtype)
            fl = 2.0 * B * hw * hw * cin * cout * 9
            t = timeit(lambda: C.conv_fwd_raw(x, wf, bg, y, B, hw, hw, spec.cin_p, spec.cout_p, cout, out_ps=ps,
                                              out_nchw=spec.out_nchw))
            res.append(dict(v=variant, k='fwd', cin=cin, cout=cout, hw=hw, ms=t, tflops=fl / t / 1e9))
            if spec.out_nchw:
                dy = torch.randn(B, hw, hw, spec.cout_p, device=dev).to(dtype)
                psx = 0
            else:
                dy = torch.randn(shp, device=dev).to(dtype)
                psx = ps
            dx = torch.empty(B, hw, hw, spec.cin_p, device=dev, dtype=dtype)
            t = timeit(lambda: C.conv_fwd_raw(dy, wd, None, dx, B, hw, hw, spec.cout_p, spec.cin_p, spec.cin_p,
                                              in_ps=psx, ldx=dy.shape[-1]))
            res.append(dict(v=variant, k='dgrad', cin=cin, cout=cout, hw=hw, ms=t, tflops=fl / t / 1e9))
            t = timeit(lambda: C.conv_wgrad_raw(dy, x, B, hw, hw, spec.cin_p, cin, spec.cout_p, cout, out_ps=psx))
            res.append(dict(v=variant, k='wgrad', cin=cin, cout=cout, hw=hw, ms=t, tflops=fl / t / 1e9))
    for r in res:
        print(json.dumps(r))


if __name__ == '__main__':
    main()
