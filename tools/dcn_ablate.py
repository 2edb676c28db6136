"""Ablations of the windowed fused DCN forward at the C5 op config (GPU box): kernel-only time
(HIP events around back-to-back sr_dcn_fwd_fused calls) for the SR_DCN_DBG masks / SR_DCN_R radii knobs,
then the op's fwd time.  Usage: python tools/dcn_ablate.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from basicsr4rs_amd import _lib  # noqa: E402
from basicsr4rs_amd.ops import dcn as D  # noqa: E402
from tools.bench_dcn import inputs  # noqa: E402


def main():
    dev = torch.device('cuda')
    x, off, msk, w, b, _ = inputs(16, dev)
    g = D._Geom(x, w, 1, 1, 1, 1, 8)
    lib = _lib.load()
    xh = D.C.nchw_to_nhwc(x, g.Cp, torch.bfloat16)
    wf, _, bg = D._prepared(w, b, g, D._spec(g), torch.bfloat16)[0]
    y = torch.empty(g.N, g.cout, g.Ho, g.Wo, device=dev)
    cols = torch.empty(g.N, g.Ho, g.Wo, g.L, device=dev, dtype=torch.bfloat16)

    def run(c):
        _lib.check(lib.sr_dcn_fwd_fused(g.desc(torch.bfloat16), _lib.ptr(xh), 0, _lib.ptr(off), _lib.ptr(msk),
                                        _lib.ptr(wf), wf.shape[1], wf.shape[0], g.cout, _lib.ptr(bg), _lib.ptr(y),
                                        _lib.ptr(c), _lib.stream()))

    def t(c=None, it=20):
        for _ in range(3):
            run(c)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(it):
            run(c)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / it * 1e3

    if os.environ.get('RS') == 'none':  # the plain kernel only (PMC passes): fwd, then fwd + cols
        print(f'fwd {t(it=5):.1f} us, with cols {t(cols, it=5):.1f} us')
        return
    from basicsr4rs_amd import _lib
    for r in (os.environ.get('RS') or '2 3 4 1 0').split():
        for dbg in (0, 1, 2, 4, 8, 3, 7, 15):
            with _lib.knob('SR_DCN_R', int(r)), _lib.knob('SR_DCN_DBG', dbg):  # library knobs (sr_set_knob)
                print(f'R {r} dbg {dbg:2d}: {t():7.1f} us' + (f'   with cols {t(cols):7.1f} us' if dbg == 0 else ''),
                      flush=True)


if __name__ == '__main__':
    main()
