"""Run-to-run determinism of a workload's train step: the same seeded model and batch trained for
--steps steps, --repeats times in one process; prints each run's loss trajectory and whether the
runs agree bitwise (losses and a parameter checksum).

usage (GPU box): python tools/determinism.py --workload swinir --steps 6 --repeats 3 [--batch 32]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def one_run(workload, steps, batch, graph, dev):
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    torch.manual_seed(42)
    wl = bench.WORKLOADS[workload]
    B = batch or wl[3]
    use_graph = bench.GRAPH_DEFAULT.get(workload, True) if graph < 0 else bool(graph)
    model = build_model(bench.make_opt(1, B, workload, use_graph))
    g0 = torch.Generator(device=dev).manual_seed(0)
    g1 = torch.Generator(device=dev).manual_seed(1)
    lq = torch.rand(B, 3, wl[4], wl[4], generator=g0, device=dev)
    gt = torch.rand(B, 3, 4 * wl[4], 4 * wl[4], generator=g1, device=dev)
    model.feed_data({'lq': lq, 'gt': gt})
    losses, grads = [], []
    for it in range(1, steps + 1):
        model.update_learning_rate(it)
        model.optimize_parameters(it)
        torch.cuda.synchronize()
        losses.append(model.get_current_log().get('l_pix'))
        grads.append({n: p.grad.detach().clone().cpu() for n, p in model.net_g.named_parameters() if p.grad is not None})
    csum = sum(float(p.detach().double().sum()) for p in model.net_g.parameters())
    del model
    torch.cuda.synchronize()
    return losses, csum, grads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='swinir')
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--repeats', type=int, default=3)
    ap.add_argument('--batch', type=int, default=0)
    ap.add_argument('--graph', type=int, default=-1)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    runs = [one_run(args.workload, args.steps, args.batch, args.graph, dev) for _ in range(args.repeats)]
    same = all(r[:2] == runs[0][:2] for r in runs[1:])
    for i, (ls, cs, _) in enumerate(runs):
        print(json.dumps({'run': i, 'losses': ls, 'param_sum': cs}))
    # the first step whose gradients differ between runs, and the parameters that differ there
    for r in range(1, len(runs)):
        for st, (ga, gb) in enumerate(zip(runs[0][2], runs[r][2])):
            bad = [n for n in ga if not torch.equal(ga[n], gb[n])]
            if bad:
                print(json.dumps({'run': r, 'first_step_differing': st + 1, 'n_params': len(bad), 'params': bad[:40]}))
                break
    print(json.dumps({'workload': args.workload, 'deterministic': same}))
    sys.exit(0 if same else 1)


if __name__ == '__main__':
    main()
