"""Halo forward variants vs the default selection on the RRDB dense shapes: max |diff| and whether
bitwise equal (a different K order rounds differently).  usage: python tools/halo_variant_check.py V[,V..]"""
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd import _lib  # noqa: E402
from basicsr4rs_amd.ops import conv as C  # noqa: E402


def main():
    variants = [int(v) for v in sys.argv[1].split(',')]
    lib = _lib.load()
    torch.manual_seed(0)
    for cin, cout, ldx in ((64, 32, 224), (96, 32, 224), (160, 32, 224), (40, 32, 224), (192, 64, 192), (32, 64, 32)):
        N, H, W = 2, 16, 128
        w = torch.randn(cout, cin, 3, 3, device='cuda') * 0.05
        b = torch.randn(cout, device='cuda') * 0.1
        wf, _, bg = C.prepared(w, b, C.ConvSpec(cin, cout), torch.bfloat16)
        xw = torch.randn(N, H, W, ldx, device='cuda').to(torch.bfloat16)
        outs = []
        for v in [0] + variants:
            _lib.check(lib.sr_conv3x3_set_variant(v))
            y = torch.zeros(N, H, W, cout, device='cuda', dtype=torch.bfloat16)
            C.conv_fwd_raw(xw, wf, bg, y, N, H, W, cin, cout, cout, ldx=ldx, xcoff=8, act=_lib.ACT_LRELU,
                           slope=0.2)
            outs.append(y)
        _lib.check(lib.sr_conv3x3_set_variant(0))
        torch.cuda.synchronize()
        for v, o in zip(variants, outs[1:]):
            print(v, cin, cout, 'equal' if torch.equal(outs[0], o) else
                  'max|diff| %.3e of %.3e' % ((outs[0].float() - o.float()).abs().max().item(),
                                             outs[0].float().abs().max().item()), flush=True)


if __name__ == '__main__':
    main()
