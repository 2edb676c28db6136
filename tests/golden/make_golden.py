"""Generates the golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference holds no golden vectors for the hot path and its Python may
not be executed here, so these fixtures pin the oracle (and, through the GPU parity tests,
the HIP engine) against regressions: inputs U[0,1) seed 0, weights from the arch's own
init with seed 42, fp32, single-threaded CPU.  Run: python -m tests.golden.make_golden
"""
import os

import numpy as np
import torch

from oracle import nets as O

CASES = {
    'edsr_tiny': dict(arch=dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=32, num_block=2, upscale=4,
                                res_scale=0.1), x=(1, 3, 16, 16), fn='edsr',
                      kw=dict(num_block=2, upscale=4, res_scale=0.1)),
    'msrresnet_tiny': dict(arch=dict(type='MSRResNet', num_in_ch=3, num_out_ch=3, num_feat=16, num_block=2,
                                     upscale=4), x=(1, 3, 12, 12), fn='msrresnet', kw=dict(num_block=2, upscale=4)),
    'rcan_tiny': dict(arch=dict(type='RCAN', num_in_ch=3, num_out_ch=3, num_feat=32, num_group=2, num_block=2,
                                squeeze_factor=16, upscale=2), x=(1, 3, 12, 12), fn='rcan',
                      kw=dict(num_group=2, num_block=2, upscale=2)),
    'rrdb_tiny': dict(arch=dict(type='RRDBNet', num_in_ch=3, num_out_ch=3, scale=4, num_feat=16, num_block=2,
                                num_grow_ch=8), x=(1, 3, 8, 8), fn='rrdbnet', kw=dict(scale=4, num_block=2)),
    'swinir_tiny': dict(arch=dict(type='SwinIR', upscale=2, in_chans=3, img_size=16, window_size=4, img_range=1.,
                                  depths=[2], embed_dim=24, num_heads=[2], mlp_ratio=2, upsampler='pixelshuffle',
                                  drop_path_rate=0.), x=(1, 3, 16, 16), fn='swinir', kw={}),
}


def run_case(case, sd, x):
    fn = getattr(O, case['fn'])
    kw = dict(case['kw'])
    if case['fn'] == 'swinir':
        kw['cfg'] = case['arch']
    with torch.no_grad():
        return fn(sd, x, **kw)


def main():
    from basicsr4rs_amd.archs import build_network
    from basicsr4rs_amd.utils.registry import ARCH_REGISTRY
    torch.set_num_threads(1)
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name, case in CASES.items():
        if case['arch']['type'] not in ARCH_REGISTRY or not hasattr(O, case['fn']):
            print('skip', name)
            continue
        torch.manual_seed(42)
        net = build_network(case['arch'])
        sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
        x = torch.rand(*case['x'], generator=torch.Generator().manual_seed(0))
        y = run_case(case, sd, x)
        arrays = {f'sd.{k}': v.numpy() for k, v in sd.items()}
        np.savez_compressed(os.path.join(out_dir, f'{name}.npz'), x=x.numpy(), y=y.numpy(), **arrays)
        print(name, tuple(y.shape), os.path.getsize(os.path.join(out_dir, f'{name}.npz')))


if __name__ == '__main__':
    main()
