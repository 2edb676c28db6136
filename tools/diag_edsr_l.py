import copy, sys, torch
sys.path.insert(0, '.')
from oracle import nets as O
from basicsr4rs_amd.archs import build_network
EDSR_L = dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=256, num_block=32, upscale=4, res_scale=0.1,
              img_range=255., rgb_mean=[0.4488, 0.4371, 0.4040])
cuda = torch.device('cuda')
torch.manual_seed(0)
net = build_network(dict(EDSR_L))
sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
H = int(sys.argv[1]) if len(sys.argv) > 1 else 48
x = torch.rand(1, 3, H, H, generator=torch.Generator().manual_seed(1))
res = {}
for dt in (torch.float32, torch.float64):
    sdg = {k: v.clone().to(dt).requires_grad_(True) for k, v in sd.items()}
    ref = O.edsr(sdg, x.to(dt), num_block=32, upscale=4, res_scale=0.1)
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(2)).to(dt)
    (ref * g).sum().backward()
    res[dt] = (ref.detach(), {k: v.grad for k, v in sdg.items()}, g)
gn = copy.deepcopy(net).to(cuda)
out = gn(x.to(cuda))
(out * res[torch.float32][2].to(cuda)).sum().backward()
r32, g32, _ = res[torch.float32]; r64, g64, _ = res[torch.float64]
print('out err gpu-64', (out.detach().cpu().double() - r64).abs().max().item(), 'cpu32-64', (r32.double() - r64).abs().max().item())
for n, p in gn.named_parameters():
    a = g64[n]; m = a.abs().max().item()
    eg = (p.grad.cpu().double() - a).abs().max().item() / m
    ec = (g32[n].double() - a).abs().max().item() / m
    if eg > 1e-4 or ec > 1e-4:
        print(f'{n:30s} gpu {eg:.2e} cpu32 {ec:.2e} max {m:.2e}')
