"""Dump weight gradients of the 256x256 wgrad kernel at the EDSR-L shapes (body conv, grouped bias;
upsample conv with pixel-shuffled dy, fused bias; a partial last K-step) for a bitwise comparison of
two library builds: SR_HIP_LIB=<lib> python tools/wgrad_dump.py out.pt; python tools/wgrad_dump.py --cmp a.pt b.pt"""
import sys

import torch

sys.path.insert(0, '.')


def main():
    if sys.argv[1] == '--cmp':
        a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        print('bitwise equal' if not bad else f'DIFFER: {bad}')
        sys.exit(1 if bad else 0)
    from basicsr4rs_amd.ops import conv as C
    dev = 'cuda'
    out = {}
    for name, (N, H, W, cin, cout, ps) in {'body': (32, 64, 64, 256, 256, 0), 'ups': (8, 64, 64, 256, 1024, 2),
                                           'ragged': (3, 20, 64, 256, 256, 0)}.items():
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.randn(N, H, W, cin, device=dev, generator=g).to(torch.bfloat16)
        r = ps if ps else 1
        dy = torch.randn(N, H * r, W * r, cout // (r * r), device=dev, generator=g).to(torch.bfloat16)
        dw, db = C.conv_wgrad_raw(dy, x, N, H, W, cin, cin, cout, cout, out_ps=ps)
        torch.cuda.synchronize()
        out[name + '_w'], out[name + '_b'] = dw.cpu(), db.cpu()
        print(name, C._lib.load().sr_conv3x3_wgrad_kernel_name(C._lib.WgradDesc()).decode() if False else '', flush=True)
    torch.save(out, sys.argv[1])


if __name__ == '__main__':
    main()
