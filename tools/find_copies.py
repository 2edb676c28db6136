"""Where the device copies of a train step come from (GPU box): two eager steps of a bench workload
under torch.profiler (CPU activity, Python stacks); prints the aten copy-like ops grouped by the
innermost basicsr4rs_amd frame.  Usage: python tools/find_copies.py [workload]"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else 'rcan'
    import basicsr4rs_amd.archs  # noqa: F401
    from basicsr4rs_amd.models import build_model
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    w = bench.WORKLOADS[wl]
    B = int(os.environ.get('B', w[3]))
    opt = bench.make_opt(1, B, wl, False)
    opt['rank'] = 0
    model = build_model(opt)
    lq = torch.rand(B, 3, w[4], w[4], device=dev)
    gt = torch.rand(B, 3, 4 * w[4], 4 * w[4], device=dev)
    model.feed_data({'lq': lq, 'gt': gt})
    for it in (1, 2):
        model.optimize_parameters(it)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        model.optimize_parameters(3)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.name in ('aten::copy_', 'aten::clone', 'aten::contiguous', 'aten::to', 'aten::_to_copy', 'aten::cat',
                       'aten::zeros', 'aten::zero_', 'aten::fill_', 'aten::add_', 'aten::add', 'aten::mul'):
            st = [f for f in (ev.stack or []) if 'basicsr4rs_amd' in f or 'bench' in f]
            where = st[0] if st else '(no repo frame: ' + ' <- '.join((ev.stack or ['?'])[:3]) + ')'
            cnt[(ev.name, where + f' shapes={ev.input_shapes} types={getattr(ev, "input_types", None)}')] += 1
    for (name, where), c in cnt.most_common(40):
        print(f'{c:5d}  {name:18s} {where}')
    # device-side copies / fills and the CPU op that issued them
    dev = collections.Counter()
    for ev in prof.events():
        for k in getattr(ev, 'kernels', []) or []:
            if any(t in k.name for t in ('opy', 'emcpy', 'ill')):
                st = [f for f in (ev.stack or []) if 'basicsr4rs_amd' in f or 'bench' in f]
                dev[(k.name[:60], ev.name, st[0] if st else '?', str(ev.input_shapes)[:80])] += 1
    for (kn, op, where, sh), c in dev.most_common(30):
        print(f'{c:5d}  {kn:40s} <- {op} {where} {sh}')


if __name__ == '__main__':
    main()
