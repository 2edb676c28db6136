"""Probe: time the stock PyTorch (MIOpen) EDSR_Lx4 train step on this GPU.

This is the reference's own execution strategy (torch nn.Conv2d + autocast) run on
MI355X, used only as a comparison point for our HIP engine. Not part of the product.
"""
import json, sys, time, torch, torch.nn as nn

def edsr_l(nf=256, nb=32, rs=0.1):
    class RB(nn.Module):
        def __init__(s):
            super().__init__(); s.c1 = nn.Conv2d(nf, nf, 3, 1, 1); s.c2 = nn.Conv2d(nf, nf, 3, 1, 1)
        def forward(s, x):
            return x + s.c2(torch.relu(s.c1(x))) * rs
    class Net(nn.Module):
        def __init__(s):
            super().__init__()
            s.head = nn.Conv2d(3, nf, 3, 1, 1); s.body = nn.Sequential(*[RB() for _ in range(nb)])
            s.cab = nn.Conv2d(nf, nf, 3, 1, 1)
            s.up = nn.Sequential(nn.Conv2d(nf, 4 * nf, 3, 1, 1), nn.PixelShuffle(2), nn.Conv2d(nf, 4 * nf, 3, 1, 1), nn.PixelShuffle(2))
            s.last = nn.Conv2d(nf, 3, 3, 1, 1)
        def forward(s, x):
            x = s.head(x); r = s.cab(s.body(x)) + x
            return s.last(s.up(r))
    return Net()

def main():
    dev = 'cuda'
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    cl = (sys.argv[2] == 'cl') if len(sys.argv) > 2 else True
    torch.backends.cudnn.benchmark = True
    net = edsr_l().to(dev)
    if cl: net = net.to(memory_format=torch.channels_last)
    opt = torch.optim.Adam(net.parameters(), 1e-4, betas=(0.9, 0.99))
    x = torch.rand(B, 3, 64, 64, device=dev); y = torch.rand(B, 3, 256, 256, device=dev)
    if cl: x = x.to(memory_format=torch.channels_last)
    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = net(x)
        loss = (out.float() - y).abs().mean(); loss.backward(); opt.step()
    for _ in range(3): step()
    torch.cuda.synchronize(); t = time.time(); n = 5
    for _ in range(n): step()
    torch.cuda.synchronize(); dt = (time.time() - t) / n
    print(json.dumps({"probe": "torch_miopen_edsr_l", "B": B, "channels_last": cl, "ms_per_step": dt * 1e3,
                      "hr_px_per_s": B * 256 * 256 / dt, "tflops": 3 * 411.7e9 * B / dt / 1e12}))
    # single conv timings
    for (ci, co, hw) in [(256, 256, 64), (256, 1024, 64), (256, 1024, 128)]:
        conv = nn.Conv2d(ci, co, 3, 1, 1).to(dev).to(torch.bfloat16)
        xi = torch.randn(B, ci, hw, hw, device=dev, dtype=torch.bfloat16)
        if cl: conv = conv.to(memory_format=torch.channels_last); xi = xi.to(memory_format=torch.channels_last)
        for _ in range(3): conv(xi)
        torch.cuda.synchronize(); t = time.time()
        for _ in range(10): conv(xi)
        torch.cuda.synchronize(); dt = (time.time() - t) / 10
        fl = 2 * B * hw * hw * co * ci * 9
        print(json.dumps({"conv": [ci, co, hw], "ms": dt * 1e3, "tflops": fl / dt / 1e12}))

if __name__ == '__main__':
    main()
