import sys
import torch
sys.path.insert(0, '.')
from torch import nn
from basicsr4rs_amd import _lib
from basicsr4rs_amd.ops import conv as C
lib = _lib.load()
N, H, W, cin, cout = [int(v) for v in sys.argv[1].split(',')]
torch.manual_seed(4)
dt = torch.bfloat16
conv = nn.Conv2d(cin, cout, 3, 1, 1).cuda()
wf, wd, bg = C.prepared(conv.weight, conv.bias, C.ConvSpec(cin, cout), dt)
x = torch.randn(N, H, W, cin, device='cuda').to(dt)
outs = []
for v in (0, 34):
    C._lib.check(lib.sr_conv3x3_set_variant(v))
    y = torch.zeros(N, H, W, cout, device='cuda', dtype=dt)
    C.conv_fwd_raw(x, wf, bg, y, N, H, W, cin, cout, cout)
    outs.append(y.float())
d = (outs[0] - outs[1]).abs()
print('maxdiff', d.max().item())
bad = (d > 1e-2)
print('bad per row y', bad.any(-1).any(-1).any(0).nonzero().flatten().tolist())
print('bad per x', bad.any(-1).any(1).any(0).nonzero().flatten().tolist()[:70])
print('bad per ch', bad.any(0).any(0).any(0).nonzero().flatten().tolist())
print('band zero?', outs[0].abs().max().item(), outs[1].abs().max().item())
