"""Fused SwinIR attention / MLP halves (csrc/swin_fused.hip) at the C4 bench shape (SwinIR-M, B 32,
64x64 tokens, embed 180): HIP-event time per launch, train and inference, for each value of the
timing-ablation knob SR_SWIN_ATTN_DBG given on the command line (0 = the kernel; others give wrong
results: 1 no step-A MFMAs, 2 no softmax VALU, 4 no step-C MFMAs, 8 no LayerNorm math, 16 no weight
staging).  usage: python tools/bench_swin_fused.py [dbg,dbg,...]"""
import json
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from basicsr4rs_amd import _lib  # noqa: E402


def main():
    dbgs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '0').split(',')]
    from basicsr4rs_amd.archs import build_network
    from basicsr4rs_amd.ops import swin as S
    cfg = bench.WORKLOADS['swinir'][0]
    torch.manual_seed(0)
    net = build_network(dict(cfg)).cuda()

    class _M:  # bench.swin_fused_roofline takes a model with get_bare_model
        net_g = net

        @staticmethod
        def get_bare_model(n):
            return n
    for d in dbgs:
        with _lib.knob('SR_SWIN_ATTN_DBG', d):
            r = bench.swin_fused_roofline(_M, 32, 64, 'cuda', reps=30)
        print(json.dumps({'dbg': d, **{k: v for k, v in r.items() if isinstance(v, dict)}}), flush=True)


if __name__ == '__main__':
    main()
