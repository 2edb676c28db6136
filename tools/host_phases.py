"""Host vs device time per phase of the eager train step (SwinIR-M by default): for a few steps,
host perf_counter stamps and device events at: step start, forward issued, backward issued
(l_total.backward() returned, side stream joined), optimizer issued.  A phase whose host time
exceeds its device time leaves the GPU waiting for launches.
Usage: python tools/host_phases.py [--workload swinir] [--steps 5]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from basicsr4rs_amd.models import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--workload', default='swinir')
ap.add_argument('--steps', type=int, default=5)
args = ap.parse_args()
dev = torch.device('cuda:0')
wl = bench.WORKLOADS[args.workload]
B, lr_px = wl[3], wl[4]
model = build_model(bench.make_opt(1, B, args.workload, False))
lq = torch.rand(B, 3, lr_px, lr_px, device=dev)
gt = torch.rand(B, 3, 4 * lr_px, 4 * lr_px, device=dev)
model.feed_data({'lq': lq, 'gt': gt})
stamps = []
orig_fwd = model.net_g.forward


def fwd(*a, **k):
    y = orig_fwd(*a, **k)
    stamps.append(('forward', time.perf_counter(), torch.cuda.Event(enable_timing=True)))
    stamps[-1][2].record()
    return y


model.net_g.forward = fwd
orig_bwd = torch.Tensor.backward


def bwd(self, *a, **k):
    r = orig_bwd(self, *a, **k)
    return r


for it in range(3 + args.steps):
    if it == 3:
        torch.cuda.synchronize()
        stamps.clear()
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    stamps.append(('start', time.perf_counter(), e))
    model.optimize_parameters(it + 1)
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    stamps.append(('end', time.perf_counter(), e))
torch.cuda.synchronize()
for i in range(len(stamps) - 1):
    (n0, h0, e0), (n1, h1, e1) = stamps[i], stamps[i + 1]
    if n0 == 'end':
        continue
    print(f'{n0:>8} -> {n1:<8} host {1e3 * (h1 - h0):7.2f} ms   device {e0.elapsed_time(e1):7.2f} ms')
