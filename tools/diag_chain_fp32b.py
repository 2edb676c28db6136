"""Diagnostic: intermediate gradients of the RRDB tail in fp32 (per-conv path) against fp64."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from tests import test_hr_tail_gpu as T
from basicsr4rs_amd.ops import conv as C

convs = T._tail(5)
torch.manual_seed(6)
feat = torch.randn(2, 24, 40, T.NF, device='cuda')
g = torch.randn(2, 3, 96, 160, device='cuda')
# GPU per-conv path with hooks on the intermediate maps
acts, grads = [], {}
x = feat.clone().requires_grad_(True)
y = x
for i, (c, kw) in enumerate(zip(convs, T.KWS)):
    y = C.conv3x3(y, c, **kw)
    if i < 3:
        acts.append(y)
        y.register_hook(lambda gr, i=i: grads.__setitem__(i, gr.detach().clone()))
y.backward(g)
torch.cuda.synchronize()
# fp64 reference with retained intermediates
xd = feat.detach().permute(0, 3, 1, 2).double()
ws = [(c.weight.detach().double(), c.bias.detach().double()) for c in convs]
h1 = F.leaky_relu(F.conv2d(F.interpolate(xd, scale_factor=2, mode='nearest'), *ws[0], padding=1), 0.2)
h2 = F.leaky_relu(F.conv2d(F.interpolate(h1, scale_factor=2, mode='nearest'), *ws[1], padding=1), 0.2)
h3 = F.leaky_relu(F.conv2d(h2, *ws[2], padding=1), 0.2)
hs = [h1, h2, h3]
for h in hs:
    h.requires_grad_(True)
    h.retain_grad()
yr = F.conv2d(hs[2], *ws[3], padding=1)
yr.backward(g.double())
# grads wrt h3 only (h1, h2 detached): recompute the chain for h2 / h1 separately
def rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()
print('act rel', [rel(acts[i].permute(0, 3, 1, 2), hs[i].detach()) for i in range(3)])
print('grad h3 rel', rel(grads[2].permute(0, 3, 1, 2), hs[2].grad))
h2b = hs[1].detach().requires_grad_(True)
h3b = F.leaky_relu(F.conv2d(h2b, *ws[2], padding=1), 0.2)
(F.conv2d(h3b, *ws[3], padding=1) * g.double()).sum().backward()
print('grad h2 rel', rel(grads[1].permute(0, 3, 1, 2), h2b.grad))
z3 = F.conv2d(hs[1].detach(), *ws[2], padding=1)
print('|z3| small count', (z3.abs() < 1e-5).sum().item(), 'of', z3.numel(), 'sign mismatch',
      ((acts[2].permute(0, 3, 1, 2).double() > 0) != (z3 > 0)).sum().item())
print('act3 dtype', acts[2].dtype, 'grad3 dtype', grads[2].dtype)
