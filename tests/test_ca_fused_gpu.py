"""The fused RCAB channel-attention kernels (csrc/blocks.hip: sr_ca_fwd_apply, sr_ca_bwd_apply,
sr_ca_param_grad) against a float64 torch restatement of ChannelAttention + the RCAB tail
(basicsr/archs/rcan_arch.py:8-24, :44-46):

    pool = mean_p u,  h = relu(W1 pool + b1),  s = sigmoid(W2 h + b2),  y = x + rs * u * s

and its backward for a given dy: du, dW1, db1, dW2, db2.  The kernels take the pooled sums as P
partial rows per image (the conv epilogue's colsum / sr_channel_partials), so the partial rows are
built here from the same u (or dy * u) split into P pixel chunks.  fp32: relative 1e-5; bf16 maps:
within bf16 rounding of the stored outputs (2^-8 relative)."""
import pytest
import torch

from basicsr4rs_amd import _lib

pytestmark = pytest.mark.gpu


def _parts(a, P):
    N, H, W, C = a.shape
    return a.reshape(N, P, (H * W) // P, C).double().sum(2).float().contiguous()


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('N,H,W,C,Cr,P', [(3, 16, 16, 64, 4, 16), (2, 64, 64, 64, 4, 128), (2, 8, 12, 32, 2, 1)])
def test_ca_fused_fwd_bwd(cuda, dtype, N, H, W, C, Cr, P):
    g = torch.Generator().manual_seed(N * 1000 + C)
    x = torch.randn(N, H, W, C, generator=g).to(dtype)
    u = torch.randn(N, H, W, C, generator=g).to(dtype)
    dy = torch.randn(N, H, W, C, generator=g).to(dtype)
    w1, b1 = torch.randn(Cr, C, generator=g) * 0.2, torch.randn(Cr, generator=g) * 0.1
    w2, b2 = torch.randn(C, Cr, generator=g) * 0.2, torch.randn(C, generator=g) * 0.1
    rs = 0.7
    # float64 reference on the same (rounded) maps
    xd, ud, dyd = x.double(), u.double(), dy.double()
    W1, B1, W2, B2 = (t.double().requires_grad_(True) for t in (w1, b1, w2, b2))
    ud.requires_grad_(True)
    pool = ud.mean((1, 2))
    hh = torch.relu(pool @ W1.t() + B1)
    ss = torch.sigmoid(hh @ W2.t() + B2)
    y = xd + rs * ud * ss[:, None, None, :]
    y.backward(dyd)
    lib = _lib.load()
    dev = lambda t: t.contiguous().to(cuda)  # noqa: E731
    xg, ug, dyg = dev(x), dev(u), dev(dy)
    w1g, b1g, w2g, b2g = dev(w1), dev(b1), dev(w2), dev(b2)  # held: the launches read them asynchronously
    parts = dev(_parts(u.float(), P))
    yo = torch.empty_like(xg)
    po = torch.empty(N, C, device=cuda)
    ho = torch.empty(N, Cr, device=cuda)
    so = torch.empty(N, C, device=cuda)
    _lib.check(lib.sr_ca_fwd_apply(_lib.dtype_code(dtype), _lib.ptr(parts), P, 1.0 / (H * W), _lib.ptr(w1g),
                                   _lib.ptr(b1g), _lib.ptr(w2g), _lib.ptr(b2g), _lib.ptr(xg), _lib.ptr(ug),
                                   N, H * W, C, Cr, rs, _lib.ptr(yo), _lib.ptr(po), _lib.ptr(ho), _lib.ptr(so),
                                   _lib.stream()))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert torch.allclose(po.cpu().double(), pool.detach(), rtol=1e-5, atol=1e-5)
    assert torch.allclose(so.cpu().double(), ss.detach(), rtol=1e-5, atol=1e-6)
    assert torch.allclose(ho.cpu().double(), hh.detach(), rtol=1e-5, atol=1e-5)
    assert (yo.float().cpu().double() - y.detach()).abs().max().item() <= tol * max(1.0, y.abs().max().item())
    # backward: parts of dy * u, then du and the per-image dz2 / dz1, then the parameter gradients
    pdu = dev(_parts((dy.float() * u.float()), P))
    du = torch.empty_like(dyg)
    dz2 = torch.empty(N, C, device=cuda)
    dz1 = torch.empty(N, Cr, device=cuda)
    _lib.check(lib.sr_ca_bwd_apply(_lib.dtype_code(dtype), _lib.ptr(pdu), P, rs, _lib.ptr(so), _lib.ptr(ho),
                                   _lib.ptr(w1g), _lib.ptr(w2g), _lib.ptr(dyg), N, H * W, C, Cr, _lib.ptr(du),
                                   _lib.ptr(dz2), _lib.ptr(dz1), _lib.stream()))
    ref_du = ud.grad
    assert (du.float().cpu().double() - ref_du).abs().max().item() <= tol * max(1.0, ref_du.abs().max().item())
    gw1 = torch.full((Cr, C), 0.5, device=cuda)  # accumulate = 1 adds onto what is there
    gb1 = torch.full((Cr, ), 0.5, device=cuda)
    gw2 = torch.full((C, Cr), 0.5, device=cuda)
    gb2 = torch.full((C, ), 0.5, device=cuda)
    _lib.check(lib.sr_ca_param_grad(_lib.ptr(dz2), _lib.ptr(dz1), _lib.ptr(ho), _lib.ptr(po), N, C, Cr, _lib.ptr(gw1),
                                    _lib.ptr(gb1), _lib.ptr(gw2), _lib.ptr(gb2), 1, _lib.stream()))
    for got, ref in ((gw1, W1.grad), (gb1, B1.grad), (gw2, W2.grad), (gb2, B2.grad)):
        err = (got.cpu().double() - 0.5 - ref).abs().max().item() / max(1e-3, ref.abs().max().item())
        assert err < (1e-4 if dtype == torch.float32 else 2e-2), err


def test_ca_fused_rejects_bad_shapes(cuda):
    lib = _lib.load()
    z = torch.zeros(64, device=cuda)
    rc = lib.sr_ca_fwd_apply(_lib.SR_F32, _lib.ptr(z), 1, 1.0, _lib.ptr(z), None, _lib.ptr(z), None, _lib.ptr(z), _lib.ptr(z), 1,
                             4, 12, 2, 1.0, _lib.ptr(z), _lib.ptr(z), _lib.ptr(z), _lib.ptr(z), _lib.stream())
    assert rc != 0 and b'C % 8' in lib.sr_last_error()
