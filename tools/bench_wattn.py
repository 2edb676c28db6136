"""Window-attention backward micro-bench at the SwinIR-M B32 shape (qkv [32, 64, 64, 576] bf16,
6 heads of 30 padded to 32, window 8, shift 4): HIP-event time per call of sr_window_attn_bwd for
the kernel forms selected by SR_WATTN_BWD / SR_WATTN_UPW (read per call), so one process A/Bs them.
Usage: python tools/bench_wattn.py [--iters N] [--forms v1,u4,u2,u1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from basicsr4rs_amd.ops import swin as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--iters', type=int, default=50)
ap.add_argument('--forms', default='v1,u4a,u4,u2,u1')
args = ap.parse_args()
dev = torch.device('cuda:0')
N, H, W, nH, hd = 32, 64, 64, 6, 30
C = nH * hd
g = S.AttnGeom(C, nH, 8, 4, 32)
torch.manual_seed(0)
qkv = torch.randn(N, H, W, 3 * nH * 32, device=dev).to(torch.bfloat16)
table = torch.randn(225, nH, device=dev) * 0.5
dout = torch.randn(N, H, W, nH * 32, device=dev).to(torch.bfloat16)
scale = hd**-0.5
out, lse = S.window_attn(qkv, g, N, H, W, scale, table)
# algorithmic bytes per call: qkv, out, dout, lse read; dqkv written (bf16, padded heads as stored)
nbytes = 2 * (2 * qkv.numel() + out.numel() + dout.numel()) + 4 * lse.numel()
for form in args.forms.split(','):
    os.environ['SR_WATTN_BWD'] = '1' if form == 'v1' else '2'
    os.environ['SR_WATTN_UPW'] = '4' if form == 'v1' else form[1:2]
    # 'a' suffix: the bias gradient by LDS atomics into 225-bin rows instead of per-lane slot rows
    os.environ['SR_WATTN_DBIAS'] = 'atomic' if form.endswith('a') else 'slots'

    for _ in range(3):
        S.window_attn_bwd(qkv, out, dout, lse, g, N, H, W, scale, table)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(args.iters):
        S.window_attn_bwd(qkv, out, dout, lse, g, N, H, W, scale, table)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.iters
    print(f'{form}: {us:.1f} us per call (incl. the dbias reduce), {nbytes / us / 1e3:.0f} GB/s algorithmic', flush=True)
