"""Compares conv_wgrad_raw under a kernel variant with variant 0 (fp32 sums in another order:
relative tolerance), at the EDSR-L wgrad shapes.  usage: python tools/wg_variant_check.py 51,52"""
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd.ops import conv as C  # noqa: E402


def main():
    lib = C._lib.load()
    torch.manual_seed(0)
    B = 32
    for v in [int(s) for s in sys.argv[1].split(',')]:
        for cin, cout, hw, ps in [(256, 256, 64, 0), (256, 1024, 64, 2), (256, 256, 48, 0)]:
            x = torch.randn(B, hw, hw, cin, device='cuda').bfloat16()
            dy = torch.randn(B, hw * (ps or 1), hw * (ps or 1), cout // max(ps, 1) ** 2, device='cuda').bfloat16()
            C._lib.check(lib.sr_conv3x3_set_variant(0))
            w0, b0 = C.conv_wgrad_raw(dy, x, B, hw, hw, cin, cin, cout, cout, out_ps=ps)
            C._lib.check(lib.sr_conv3x3_set_variant(v))
            w1, b1 = C.conv_wgrad_raw(dy, x, B, hw, hw, cin, cin, cout, cout, out_ps=ps)
            C._lib.check(lib.sr_conv3x3_set_variant(0))
            ew = ((w1 - w0).abs().max() / w0.abs().max()).item()
            eb = ((b1 - b0).abs().max() / b0.abs().max()).item()
            ok = ew < 1e-5 and eb < 1e-5
            print(f'variant {v} cin {cin} cout {cout} hw {hw} ps {ps}: rel err w {ew:.2e} b {eb:.2e}', 'OK' if ok else 'FAIL')
            if not ok:
                sys.exit(1)


if __name__ == '__main__':
    main()
