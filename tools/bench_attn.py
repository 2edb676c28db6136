"""Micro-benchmark of the SwinIR window-attention kernels at the C4 shape (SwinIR-M x4,
batch 32, 64x64 tokens, embed 180 = 6 heads x 30 (padded 32), window 8), HIP events.
Prints per-kernel ms, algorithmic TFLOP/s (QK^T + AV, head_dim 30) and GB/s (q,k,v,out /
q,k,v,out,dout,dqkv once each)."""
import json
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd.ops import swin as S  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    B, H, W, nH, hd, ws = 32, 64, 64, 6, 30, 8
    dev = 'cuda'
    res = []
    for shift in (0, 4):
        g = S.AttnGeom(nH * hd, nH, ws, shift, 32)
        qkv = torch.randn(B, H, W, 3 * nH * 32, device=dev).to(torch.bfloat16)
        table = torch.randn((2 * ws - 1)**2, nH, device=dev) * 0.1
        out, lse = S.window_attn(qkv, g, B, H, W, hd**-0.5, table)
        dout = torch.randn_like(out)
        fl = S.attn_flops(g, B, H, W)
        tok = B * H * W
        t = timeit(lambda: S.window_attn(qkv, g, B, H, W, hd**-0.5, table))
        res.append(dict(k='fwd', shift=shift, ms=t, tflops=fl / t / 1e9, gbs=tok * nH * 32 * 2 * 4 / t / 1e6))
        t = timeit(lambda: S.window_attn_bwd(qkv, out, dout, lse, g, B, H, W, hd**-0.5, table))
        res.append(dict(k='bwd', shift=shift, ms=t, tflops=2.5 * fl / t / 1e9, gbs=tok * nH * 32 * 2 * 8 / t / 1e6))
    for r in res:
        print(json.dumps(r))


if __name__ == '__main__':
    main()
