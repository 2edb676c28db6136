"""SwinIR-M linear dgrads at the C4 bench shape (B 32 x 64 x 64 tokens, embed 180, 6 heads): HIP-event
time per launch of each dgrad of a SwinTransformerBlock's backward (ops/swin.py _STB) with its
algorithmic HBM bytes (dY read, dX written, gate read) and FLOPs.  usage: python tools/bench_linear.py"""
import json
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd.ops import swin as S  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    N, H, W, C, nH = 32, 64, 64, 180, 6
    M = N * H * W
    dt = torch.bfloat16
    specs = {'qkv': S.qkv_spec(C, nH, 32), 'proj': S.proj_spec(C, nH, 32), 'fc1': S.plain_spec(C, 2 * C),
             'fc2': S.plain_spec(2 * C, C)}
    torch.manual_seed(0)
    for name, sp in specs.items():
        w = torch.randn(sp.cout, sp.cin, device='cuda') * 0.05
        b = torch.zeros(sp.cout, device='cuda')
        _, wd, _ = S.prepared_linear(w, b, sp, dt)
        dy = torch.randn(N, H, W, sp.cout_p, device='cuda').to(dt)
        nbytes = M * (sp.cout_p + sp.cin_p) * 2
        us = timeit(lambda: S.linear_dgrad(dy, wd, sp, N, H, W))
        fl = 2.0 * M * sp.cout_p * sp.cin_p
        print(json.dumps({'dgrad': name, 'K': sp.cout_p, 'Cout': sp.cin_p, 'us': round(us, 1),
                          'GB/s': round(nbytes / us / 1e3, 1), 'TF/s': round(fl / us / 1e6, 1)}), flush=True)
        if name == 'fc2':  # fc2 dgrad with the GELU' gate on z (hidden 360 -> 368)
            z = torch.randn(N, H, W, sp.cin_p, device='cuda').to(dt)
            us = timeit(lambda: S.linear_dgrad(dy, wd, sp, N, H, W, gate=z, gate_mode=1))
            print(json.dumps({'dgrad': 'fc2+gelu_gate', 'K': sp.cout_p, 'Cout': sp.cin_p, 'us': round(us, 1),
                              'GB/s': round((nbytes + M * sp.cin_p * 2) / us / 1e3, 1),
                              'TF/s': round(fl / us / 1e6, 1)}), flush=True)


if __name__ == '__main__':
    main()
