"""Diagnostic: per-layer errors of the RRDB tail chain in fp32 (chain vs per-conv path vs fp64)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from tests import test_hr_tail_gpu as T
from basicsr4rs_amd.ops import conv as C
from basicsr4rs_amd import _lib

convs = T._tail(5)
torch.manual_seed(6)
feat = torch.randn(2, 24, 40, T.NF, device='cuda')
g = torch.randn(2, 3, 96, 160, device='cuda')
ref = T._reference(convs, feat, g, False)
for chain in (True, False):
    y, dx, grads = T._run(convs, feat, g, chain)
    print('chain' if chain else 'per-conv', {k: f'{v:.2e}' for k, v in T._errs(y, dx, grads, ref).items()})
# conv_last dgrad alone, fp32, with and without the gate
c = convs[3]
spec = C.ConvSpec(64, 3, out_nchw=True)
_, wd, _ = C.prepared(c.weight, c.bias, spec, torch.float32)
dY = C.nchw_to_nhwc(g, spec.cout_p, torch.float32)
print('dY pad max', dY[..., 3:].abs().max().item())
N, H, W = 2, 96, 160
dx = torch.empty(N, H, W, 64, device='cuda')
lib = _lib.load()
print('kernel', lib.sr_conv3x3_fwd_kernel_name(C._desc(torch.float32, N, H, W, 8, 8, 64, 64, 64)).decode())
C.conv_fwd_raw(dY, wd, None, dx, N, H, W, spec.cout_p, spec.cin_p, spec.cin_p)
w64 = c.weight.detach().double()
refdx = F.conv_transpose2d(g.double(), w64, padding=1).permute(0, 2, 3, 1)
print('dgrad conv_last no gate rel', ((dx.double() - refdx).norm() / refdx.norm()).item())
gate = torch.randn(N, H, W, 64, device='cuda')
dx2 = torch.empty_like(dx)
C.conv_fwd_raw(dY, wd, None, dx2, N, H, W, spec.cout_p, spec.cin_p, spec.cin_p, gate=gate, gate_slope=0.2)
refg = refdx * torch.where(gate.double() > 0, 1.0, 0.2)
print('dgrad conv_last gate rel', ((dx2.double() - refg).norm() / refg.norm()).item())
