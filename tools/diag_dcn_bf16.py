"""Diagnostic: per-tensor error of the bf16 DCN path vs the oracle on bf16-rounded operands."""
import numpy as np
import torch

from basicsr4rs_amd.ops import dcn as D
from oracle import ops as O
from tests.test_ops_gpu import _dcn_inputs

case = (2, 64, 16, 16, 64, 3, 1, 1, 1, 1, 8, True)
x, off, msk, w, b, dy = _dcn_inputs(case, seed=1)
bfr = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()  # noqa: E731
xb, wb, dyb = bfr(x), bfr(w), bfr(dy)
for mode in ('fp32', 'bf16'):
    t = [torch.tensor(a, device='cuda', requires_grad=True) for a in (x, off, msk, w, b)]
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=mode == 'bf16'):
        out = D.modulated_deform_conv(*t, 1, 1, 1, 1, 8)
    out.backward(torch.tensor(dy, device='cuda'))
    xx, ww, dd = (xb, wb, dyb) if mode == 'bf16' else (x, w, dy)
    ref = O.dcn_forward(xx, off, msk, ww, b, 1, 1, 1, 1, 8)
    grads = O.dcn_backward(xx, off, msk, ww, b, 1, 1, 1, 1, 8, dd)
    for name, g, tt in zip(('out', 'x', 'offset', 'mask', 'weight', 'bias'), (ref, ) + grads, [out] + t):
        a = (tt if name == 'out' else tt.grad).detach().double().cpu().numpy()
        e = np.abs(a - g)
        i = np.unravel_index(e.argmax(), e.shape)
        print(mode, name, 'maxerr %.3e  max|ref| %.3e  at %s a=%.5f ref=%.5f  mean|err| %.2e' %
              (e.max(), np.abs(g).max(), i, a[i], g[i], e.mean()))
