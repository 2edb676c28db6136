"""Library reference points on the GPU box: hipBLASLt (torch.matmul) bf16 TF/s for the GEMM
shapes equivalent to the EDSR-L body conv (M = 32*64*64 px, K = 9*256, N = 256) and its wgrad
(M = 256, N = 2304, K = 131072), plus a square 8192^3 GEMM.  Not part of the product."""
import json

import torch


def bench(m, n, k, iters=50, ta=False):
    # ta: A given as the transpose of a [k, m] row-major map (a weight gradient dY^T X)
    a = torch.randn(k, m, device='cuda', dtype=torch.bfloat16).t() if ta else \
        torch.randn(m, k, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(k, n, device='cuda', dtype=torch.bfloat16)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        c = a @ b
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    return {'m': m, 'n': n, 'k': k, 'ta': ta, 'us': round(ms * 1e3, 1), 'tflops': round(2 * m * n * k / ms / 1e9, 1)}


if __name__ == '__main__':
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == 'swin':  # SwinIR-M linear weight gradients at B 32 (dY^T X)
        for m, n in [(552, 184), (184, 184), (360, 184), (184, 360)]:
            print(json.dumps(bench(m, n, 131072, ta=True)))
    else:
        for shp in [(131072, 256, 2304), (256, 2304, 131072), (8192, 8192, 8192), (131072, 64, 576)]:
            print(json.dumps(bench(*shp)))
