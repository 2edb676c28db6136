"""Band conv: the default selection (8 waves per block at W 128) vs variant 14 (4 waves everywhere)
on the RCAN / RRDB band shapes and epilogues: y bitwise (same K order per pixel), colsum partials
summed per image within fp32 reassociation.  usage: python tools/band8_check.py"""
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd import _lib  # noqa: E402
from basicsr4rs_amd.ops import conv as C  # noqa: E402


def run(lib, variant, shape, epi):
    N, H, W, cin, cout = shape
    g = torch.Generator(device='cuda').manual_seed(1)
    w = torch.randn(cout, cin, 3, 3, device='cuda', generator=g) * 0.05
    b = torch.randn(cout, device='cuda', generator=g) * 0.1
    wf, _, bg = C.prepared(w, b, C.ConvSpec(cin, cout), torch.bfloat16)
    x = torch.randn(N, H, W, cin, device='cuda', generator=g).to(torch.bfloat16)
    gate = torch.randn(N, H, W, cout, device='cuda', generator=g).to(torch.bfloat16)
    res = torch.randn(N, H, W, cout, device='cuda', generator=g).to(torch.bfloat16)
    kw = {}
    if epi == 'relu':
        kw = dict(act=_lib.ACT_RELU)
    elif epi == 'gate_res':
        kw = dict(gate=gate, gate_slope=0.2, alpha=0.3, res=res, beta=0.7)
    elif epi == 'rrdb_dgrad':
        kw = dict(alpha=0.2, res=res, beta=1.0, rcols=64, gate=gate, gate_slope=0.2, gate_mode=2, gcol0=cout - 32,
                  gcol1=cout)
    _lib.check(lib.sr_conv3x3_set_variant(variant))
    try:
        name = lib.sr_conv3x3_fwd_kernel_name(C._desc(torch.bfloat16, N, H, W, cin, cin, cout, cout, cout)).decode()
        assert name == 'conv3x3_fwd_band_kernel', name
        y = torch.zeros(N, H, W, cout, device='cuda', dtype=torch.bfloat16)
        if epi == 'colsum':
            y, parts = C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout, colsum=True)
            return y, parts.double().sum(1)
        C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout, **kw)
        return y, None
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))


def main():
    lib = _lib.load()
    ok = True
    for shape, epis in (((32, 64, 64, 64, 64), ('plain', 'relu', 'gate_res', 'colsum')),
                        ((16, 128, 128, 64, 64), ('plain', 'relu')),
                        ((16, 128, 128, 32, 64), ('rrdb_dgrad', 'plain')),
                        ((16, 128, 128, 64, 32), ('plain', 'relu', 'colsum')),
                        ((16, 128, 128, 32, 32), ('plain', 'gate_res'))):
        for epi in epis:
            y0, c0 = run(lib, 0, shape, epi)
            y1, c1 = run(lib, 14, shape, epi)
            torch.cuda.synchronize()
            eq = torch.equal(y0, y1)
            msg = f'{shape} {epi}: y {"equal" if eq else "DIFF %.3e" % (y0.float() - y1.float()).abs().max().item()}'
            if c0 is not None:
                ref = y0.double().sum((1, 2))
                e0 = ((c0 - ref).abs().max() / ref.abs().max()).item()
                e1 = ((c1 - ref).abs().max() / ref.abs().max()).item()
                msg += f' colsum rel err {e0:.2e} / {e1:.2e}'
                ok = ok and e1 < 1e-4
            ok = ok and eq
            print(msg, flush=True)
    print('OK' if ok else 'FAIL')
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
