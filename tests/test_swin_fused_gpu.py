"""The fused attention half of a SwinTransformerBlock (csrc/swin_fused.hip, round 4):
x2 = x + s1 * proj(WindowAttention(qkv(LN1(x)))) in one launch
(basicsr/archs/swinir_arch.py:283-314, WindowAttention :144-175).

* against the unfused HIP path (LN+qkv lin kernel, attention kernel, proj linear) on the same
  bf16 operands: both round LN1(x), q/k/v, P and the attention output to bf16 at the same points,
  so qkv / attention output / x2 agree to a couple of bf16 ulps and ln1 / mean / rstd / lse to fp32
  rounding -- the backward, which reads these, is shared;
* against the fp64 CPU oracle (oracle/nets.py window_attention_core + LayerNorm + linears) on the
  same bf16-rounded inputs and weights: within bf16 tolerance;
* geometries: SwinIR-M (C 180, 6 heads, hd 30), shifted and not, an odd window count (the block's
  second window past the end), SwinIR-light (C 60, hd 10), 3 heads of 32 with a DropPath row scale;
  inference mode (no saved tensors) writes the same x2;
* shifted and unshifted blocks (the kernel is specialised for each).
"""
import pytest
import torch

from oracle import nets as O

pytestmark = pytest.mark.gpu

GEOMS = [  # N, H, W, C, nH, shift, row_scale
    (2, 16, 16, 180, 6, 0, False),
    (2, 16, 16, 180, 6, 4, False),
    (1, 8, 24, 180, 6, 0, True),
    (2, 16, 24, 60, 6, 4, False),
    (3, 16, 16, 96, 3, 4, True),
]


def _setup(cuda, N, H, W, C, nH, shift, rsc):
    from basicsr4rs_amd.ops import conv as Cv
    from basicsr4rs_amd.ops import swin as S
    torch.manual_seed(N * 1000 + H * 10 + C + shift)
    g = S.AttnGeom(C, nH, 8, shift)
    Cp = Cv.pad8(C)
    x = torch.zeros(N, H, W, Cp)
    x[..., :C] = torch.randn(N, H, W, C)
    x = x.to(torch.bfloat16).to(cuda)
    n1w = (1 + 0.1 * torch.randn(C)).to(cuda)
    n1b = (0.1 * torch.randn(C)).to(cuda)
    qw = (torch.randn(3 * C, C) * 0.08).to(cuda)
    qb = (torch.randn(3 * C) * 0.05).to(cuda)
    pw = (torch.randn(C, C) * 0.08).to(cuda)
    pb = (torch.randn(C) * 0.05).to(cuda)
    table = (torch.randn(225, nH) * 0.5).to(cuda)
    s1 = (torch.rand(N) * 2).to(cuda) if rsc else None
    qwf, _, qbg = S.prepared_linear(qw, qb, g.qkv, torch.bfloat16)
    pwf, _, pbg = S.prepared_linear(pw, pb, g.proj, torch.bfloat16)
    scale = (C // nH)**-0.5
    return S, g, x, (n1w, n1b, qw, qb, pw, pb, table, s1, qwf, qbg, pwf, pbg, scale)


def _unfused(S, g, x, p):
    n1w, n1b, qw, qb, pw, pb, table, s1, qwf, qbg, pwf, pbg, scale = p
    N, H, W, Cp = x.shape
    fz = S.linear_ln_fwd(x, n1w, n1b, g.dim, qwf, qbg, g.qkv, N, H, W)
    if fz is not None:
        qkv, ln1, m1, r1 = fz
    else:
        ln1, m1, r1 = S.layernorm(x, n1w, n1b, g.dim)
        qkv = S.linear_fwd(ln1, qwf, qbg, g.qkv, N, H, W)
    a, lse = S.window_attn(qkv, g, N, H, W, scale, table)
    x2 = S.linear_fwd(a, pwf, pbg, g.proj, N, H, W, res=x, beta=1.0, row_scale=s1)
    return x2, ln1, m1, r1, qkv, a, lse


def _oracle(g, x, p):
    """fp64 restatement on the bf16-rounded inputs and weights (the GEMM images hold bf16)."""
    n1w, n1b, qw, qb, pw, pb, table, s1, _, _, _, _, scale = p
    C, nH = g.dim, g.nH
    xd = x[..., :C].double().cpu()
    sd = {'n.weight': n1w.double().cpu(), 'n.bias': n1b.double().cpu()}
    ln1 = O._ln(xd, sd, 'n')
    qkv = ln1 @ qw.cpu().to(torch.bfloat16).double().t() + qb.double().cpu()
    att = O.window_attention_core(qkv, nH, 8, g.shift, scale, table.double().cpu())
    proj = att @ pw.cpu().to(torch.bfloat16).double().t() + pb.double().cpu()
    if s1 is not None:
        proj = proj * s1.double().cpu().view(-1, 1, 1, 1)
    return xd + proj, proj, ln1, qkv, att


def _unpad_qkv(t, g):
    N, H, W, _ = t.shape
    return t.view(N, H, W, 3, g.nH, g.hdp)[..., :g.hd].reshape(N, H, W, 3 * g.dim)


def _unpad_heads(t, g):
    N, H, W, _ = t.shape
    return t.view(N, H, W, g.nH, g.hdp)[..., :g.hd].reshape(N, H, W, g.dim)


@pytest.mark.parametrize('geom', GEOMS)
def test_swin_attn_fused_vs_unfused_and_fp64(cuda, geom):
    N, H, W, C, nH, shift, rsc = geom
    S, g, x, p = _setup(cuda, N, H, W, C, nH, shift, rsc)
    n1w, n1b, qw, qb, pw, pb, table, s1, qwf, qbg, pwf, pbg, scale = p
    fz = S.swin_attn_fused(x, n1w, n1b, C, qwf, qbg, table, pwf, pbg, s1, g, scale, True)
    assert fz is not None, 'geometry not on the fused path'
    inf = S.swin_attn_fused(x, n1w, n1b, C, qwf, qbg, table, pwf, pbg, s1, g, scale, False)
    ref = _unfused(S, g, x, p)
    torch.cuda.synchronize()
    x2, ln1, m1, r1, qkv, a, lse = fz
    assert torch.equal(inf[0], x2)  # inference mode: the same x2, nothing else written
    assert all(t is None for t in inf[1:])
    # against the unfused HIP path: the same rounding points
    for name, got, want, tol in (('ln1', ln1, ref[1], 1e-2), ('qkv', qkv, ref[4], 2e-2), ('attn', a, ref[5], 2e-2)):
        err = (got.float() - want.float()).abs().max().item()
        assert err <= tol * want.float().abs().max().item(), (name, err)
    assert torch.allclose(m1, ref[2], rtol=1e-5, atol=1e-5) and torch.allclose(r1, ref[3], rtol=1e-4, atol=1e-5)
    assert (lse - ref[6]).abs().max().item() < 2e-3
    if C < x2.shape[-1]:
        assert x2[..., C:].abs().max().item() == 0.0  # padded channels stay exactly zero
    dx2 = (x2.float() - ref[0].float()).abs().max().item()
    # against fp64
    ox2, oproj, oln1, oqkv, oatt = _oracle(g, x, p)
    e_qkv = (_unpad_qkv(qkv, g).double().cpu() - oqkv).abs().max().item() / oqkv.abs().max().item()
    e_att = (_unpad_heads(a, g).double().cpu() - oatt).abs().max().item() / oatt.abs().max().item()
    e_x2 = (x2[..., :C].double().cpu() - ox2).abs().max().item() / oproj.abs().max().item()
    print(f'{geom}: fused-unfused x2 {dx2:.3e}; vs fp64 qkv {e_qkv:.3e} attn {e_att:.3e} x2 {e_x2:.3e}')
    assert dx2 <= 2e-2 * oproj.abs().max().item() + 1e-2
    assert e_qkv < 2e-2 and e_att < 3e-2 and e_x2 < 3e-2


MLP_GEOMS = [  # N, H, W, C, hidden, row_scale
    (2, 16, 16, 180, 360, False),
    (1, 8, 24, 180, 360, True),
    (2, 16, 24, 60, 120, False),
    (1, 16, 16, 96, 192, True),
]


@pytest.mark.parametrize('geom', MLP_GEOMS)
def test_swin_mlp_fused_vs_unfused_and_fp64(cuda, geom):
    """The fused MLP half, out = x2 + s2 * fc2(GELU(fc1(LN2(x2)))) (swinir_arch.py:322-323, Mlp :43-60):
    ln2 / z / h / out against the unfused path (LN-prologue lin kernel with GELU + aux, then the fc2
    linear with the residual) and out against fp64; inference writes the same out."""
    from basicsr4rs_amd.ops import conv as Cv
    from basicsr4rs_amd.ops import swin as S
    N, H, W, C, hid, rsc = geom
    torch.manual_seed(N * 100 + C + hid)
    Cp = Cv.pad8(C)
    x = torch.zeros(N, H, W, Cp)
    x[..., :C] = torch.randn(N, H, W, C)
    x = x.to(torch.bfloat16).to(cuda)
    n2w, n2b = (1 + 0.1 * torch.randn(C)).to(cuda), (0.1 * torch.randn(C)).to(cuda)
    f1w, f1b = (torch.randn(hid, C) * 0.08).to(cuda), (torch.randn(hid) * 0.05).to(cuda)
    f2w, f2b = (torch.randn(C, hid) * 0.06).to(cuda), (torch.randn(C) * 0.05).to(cuda)
    s2 = (torch.rand(N) * 2).to(cuda) if rsc else None
    fc1s, fc2s = S.plain_spec(C, hid), S.plain_spec(hid, C)
    f1wf, _, f1bg = S.prepared_linear(f1w, f1b, fc1s, torch.bfloat16)
    f2wf, _, f2bg = S.prepared_linear(f2w, f2b, fc2s, torch.bfloat16)
    fm = S.swin_mlp_fused(x, n2w, n2b, C, f1wf, f1bg, fc1s, f2wf, f2bg, s2, True)
    assert fm is not None, 'geometry not on the fused path'
    inf = S.swin_mlp_fused(x, n2w, n2b, C, f1wf, f1bg, fc1s, f2wf, f2bg, s2, False)
    z = torch.empty(N, H, W, fc1s.cout_p, device=cuda, dtype=torch.bfloat16)
    uf = S.linear_ln_fwd(x, n2w, n2b, C, f1wf, f1bg, fc1s, N, H, W, act=S.GELU, aux=z)
    if uf is not None:
        h, ln2, m2, r2 = uf
    else:
        ln2, m2, r2 = S.layernorm(x, n2w, n2b, C)
        h = S.linear_fwd(ln2, f1wf, f1bg, fc1s, N, H, W, act=S.GELU, aux=z)
    out = S.linear_fwd(h, f2wf, f2bg, fc2s, N, H, W, res=x, beta=1.0, row_scale=s2)
    torch.cuda.synchronize()
    fo, fln2, fm2, fr2, fz, fh = fm
    assert torch.equal(inf[0], fo) and all(t is None for t in inf[1:])
    for name, got, want in (('ln2', fln2, ln2), ('z', fz, z), ('h', fh, h), ('out', fo, out)):
        err = (got.float() - want.float()).abs().max().item()
        assert err <= 2e-2 * want.float().abs().max().item(), (name, err)
    assert torch.allclose(fm2, m2, rtol=1e-5, atol=1e-5) and torch.allclose(fr2, r2, rtol=1e-4, atol=1e-5)
    if C < Cp:
        assert fo[..., C:].abs().max().item() == 0.0
    xd = x[..., :C].double().cpu()
    t = torch.nn.functional.layer_norm(xd, (C, ), n2w.double().cpu(), n2b.double().cpu(), 1e-5)
    t = torch.nn.functional.gelu(t @ f1w.cpu().to(torch.bfloat16).double().t() + f1b.double().cpu())
    br = t @ f2w.cpu().to(torch.bfloat16).double().t() + f2b.double().cpu()
    if s2 is not None:
        br = br * s2.double().cpu().view(-1, 1, 1, 1)
    e = (fo[..., :C].double().cpu() - (xd + br)).abs().max().item() / br.abs().max().item()
    print(f'{geom}: mlp fused vs fp64 {e:.3e}')
    assert e < 3e-2
