"""Host time per train step and the GPU gap between consecutive steps, unprofiled: events on the
current stream right before and after each optimize_parameters call.  gap = end(k-1) -> start(k)
on the GPU (0 when the host runs ahead), gpu = start(k) -> end(k), host = the call's wall time.
Usage: python tools/replay_gap.py [--workload rcan] [--steps 10]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from basicsr4rs_amd.models import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--workload', default='rcan')
ap.add_argument('--steps', type=int, default=10)
args = ap.parse_args()
dev = torch.device('cuda:0')
wl = bench.WORKLOADS[args.workload]
B, lr_px = wl[3], wl[4]
graph = bench.GRAPH_DEFAULT.get(args.workload, True)
model = build_model(bench.make_opt(1, B, args.workload, graph))
model.feed_data({'lq': torch.rand(B, 3, lr_px, lr_px, device=dev),
                 'gt': torch.rand(B, 3, 4 * lr_px, 4 * lr_px, device=dev)})
for it in range(4):
    model.optimize_parameters(it + 1)
torch.cuda.synchronize()
ev, host = [], []
for it in range(args.steps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    model.optimize_parameters(it + 5)
    b.record()
    host.append(time.perf_counter() - t0)
    ev.append((a, b))
torch.cuda.synchronize()
for k, (a, b) in enumerate(ev):
    gap = ev[k - 1][1].elapsed_time(a) if k else float('nan')
    print(f'step {k}: host {1e3 * host[k]:7.3f} ms  gpu {a.elapsed_time(b):7.3f} ms  gap before {gap:7.3f} ms')
