"""Diagnostic: fp32 conv fwd / dgrad / wgrad against fp64 at the RRDB-tail shapes, with kernel names."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn as nn
import torch.nn.functional as F
from basicsr4rs_amd import _lib
from basicsr4rs_amd.ops import conv as C


def rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


torch.manual_seed(0)
lib = _lib.load()
for (N, H, W, cin, cout, up) in [(2, 96, 160, 64, 64, 1), (2, 48, 80, 64, 64, 2), (2, 24, 40, 64, 64, 2), (2, 96, 160, 64, 3, 1),
                                 (1, 16, 16, 64, 64, 1)]:
    conv = nn.Conv2d(cin, cout, 3, 1, 1).cuda()
    Ho, Wo = H * up, W * up
    x = torch.randn(N, H, W, cin, device='cuda')
    dy = torch.randn(N, Ho, Wo, cout, device='cuda')
    spec = C.ConvSpec(cin, cout, in_up=up)
    wf, wd, bg = C.prepared(conv.weight, conv.bias, spec, torch.float32)
    # forward
    y = torch.empty(N, Ho, Wo, spec.cout_p, device='cuda')
    C.conv_fwd_raw(x, wf, bg, y, N, Ho, Wo, spec.cin_p, spec.cout_p, cout, in_up=up)
    xd = x.permute(0, 3, 1, 2).double()
    if up > 1:
        xd = F.interpolate(xd, scale_factor=up, mode='nearest')
    wdb, bdb = conv.weight.detach().double(), conv.bias.detach().double()
    yr = F.conv2d(xd, wdb, bdb, padding=1).permute(0, 2, 3, 1)
    fk = lib.sr_conv3x3_fwd_kernel_name(C._desc(torch.float32, N, Ho, Wo, spec.cin_p, spec.cin_p, spec.cout_p, spec.cout_p, cout)).decode()
    # dgrad (on the upsampled grid)
    dyp = torch.zeros(N, Ho, Wo, spec.cout_p, device='cuda')
    dyp[..., :cout] = dy
    dx = torch.empty(N, Ho, Wo, spec.cin_p, device='cuda')
    C.conv_fwd_raw(dyp, wd, None, dx, N, Ho, Wo, spec.cout_p, spec.cin_p, spec.cin_p)
    dxr = F.conv_transpose2d(dy.permute(0, 3, 1, 2).double(), wdb, padding=1).permute(0, 2, 3, 1)
    dk = lib.sr_conv3x3_fwd_kernel_name(C._desc(torch.float32, N, Ho, Wo, spec.cout_p, spec.cout_p, spec.cin_p, spec.cin_p, spec.cin_p)).decode()
    # wgrad
    dw, db = C.conv_wgrad_raw(dyp, x, N, Ho, Wo, spec.cin_p, cin, spec.cout_p, cout, in_up=up)
    xg = xd.clone().requires_grad_(False)
    wv = wdb.clone().requires_grad_(True)
    bv = bdb.clone().requires_grad_(True)
    (F.conv2d(xd, wv, bv, padding=1) * dy.permute(0, 3, 1, 2).double()).sum().backward()
    torch.cuda.synchronize()
    wdesc = _lib.WgradDesc()
    print(f'N{N} {H}x{W} up{up} {cin}->{cout}: fwd {rel(y[..., :cout], yr):.2e} [{fk}]  dgrad {rel(dx[..., :cin], dxr):.2e} '
          f'[{dk}]  dw {rel(dw.reshape(wv.shape), wv.grad):.2e} db {rel(db, bv.grad):.2e}', flush=True)
