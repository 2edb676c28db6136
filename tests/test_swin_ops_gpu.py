"""Op-level parity of the SwinIR token kernels (csrc/swin.hip) against the oracle:
LayerNorm fwd/bwd (bf16 vectorised and fp32 paths) and the fused shifted-window attention
fwd/bwd (oracle.nets.window_attention_core, fp64 autograd) at the SwinIR-M geometry."""
import pytest
import torch
import torch.nn.functional as F

from basicsr4rs_amd.ops import swin as S
from oracle import nets as O

pytestmark = pytest.mark.gpu


def _pad_last(t, cp):
    return F.pad(t, (0, cp - t.shape[-1]))


@pytest.mark.parametrize('C,dtype', [(180, torch.bfloat16), (60, torch.bfloat16), (180, torch.float32),
                                     (300, torch.bfloat16)])
@pytest.mark.parametrize('with_res', [False, True])
def test_layernorm_fwd_bwd(cuda, C, dtype, with_res):
    torch.manual_seed(1)
    N, H, W = 2, 7, 13  # odd row count: partial wave / block tails
    Cp = (C + 7) // 8 * 8
    x = (torch.randn(N, H, W, C) * 2 + 0.5).to(dtype)
    dy = torch.randn(N, H, W, C).to(dtype)
    res = torch.randn(N, H, W, C).to(dtype)
    gw, gb = torch.randn(C) * 0.5 + 1, torch.randn(C) * 0.1
    xd = x.double().requires_grad_()
    gwd, gbd = gw.double().requires_grad_(), gb.double().requires_grad_()
    ref = F.layer_norm(xd, (C, ), gwd, gbd, 1e-5)
    ref.backward(dy.double())
    y, mean, rstd = S.layernorm(_pad_last(x, Cp).to(cuda).contiguous(), gw.to(cuda), gb.to(cuda), C)
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    assert (y[..., :C].double().cpu() - ref.detach()).abs().max().item() < tol * ref.abs().max().item()
    assert y[..., C:].abs().max().item() == 0 if Cp > C else True
    dx, dg, db = S.layernorm_bwd(_pad_last(dy, Cp).to(cuda).contiguous(), _pad_last(x, Cp).to(cuda).contiguous(), mean,
                                 rstd, gw.to(cuda), C,
                                 res=_pad_last(res, Cp).to(cuda).contiguous() if with_res else None)
    want = xd.grad + (res.double() if with_res else 0)
    assert (dx[..., :C].double().cpu() - want).abs().max().item() < tol * want.abs().max().item()
    assert (dg.double().cpu() - gwd.grad).abs().max().item() < tol * gwd.grad.abs().max().item() + 1e-3
    assert (db.double().cpu() - gbd.grad).abs().max().item() < tol * gbd.grad.abs().max().item() + 1e-3


def _qkv_padded(qkv, nH, hd, hdp):
    """[b,h,w,3*nH*hd] -> kernel layout [b,h,w,3*nH*hdp] (zero-padded heads)."""
    b, h, w, _ = qkv.shape
    return F.pad(qkv.view(b, h, w, 3, nH, hd), (0, hdp - hd)).reshape(b, h, w, 3 * nH * hdp)


@pytest.mark.parametrize('shift', [0, 4])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('geom', [(2, 16, 24, 6, 30, 8), (1, 8, 8, 2, 16, 8), (1, 12, 12, 3, 20, 4)])
def test_window_attention_fwd_bwd(cuda, shift, dtype, geom):
    b, h, w, nH, hd, ws = geom
    if shift >= ws // 2 + 1 or min(h, w) <= ws:
        shift = 0 if min(h, w) <= ws else ws // 2
    torch.manual_seed(2)
    C = nH * hd
    hdp = 32
    scale = hd**-0.5
    qkv = torch.randn(b, h, w, 3 * C).to(dtype)
    table = torch.randn((2 * ws - 1)**2, nH) * 0.5
    dout = torch.randn(b, h, w, C).to(dtype)
    qd = qkv.double().requires_grad_()
    td = table.double().requires_grad_()
    ref = O.window_attention_core(qd, nH, ws, shift, scale, td)
    ref.backward(dout.double())
    g = S.AttnGeom(C, nH, ws, shift, hdp)
    qp = _qkv_padded(qkv, nH, hd, hdp).to(cuda).contiguous()
    out, lse = S.window_attn(qp, g, b, h, w, scale, table.to(cuda))
    got = out.view(b, h, w, nH, hdp)[..., :hd].reshape(b, h, w, C).double().cpu()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert (got - ref.detach()).abs().max().item() < tol * max(1.0, ref.abs().max().item())
    assert out.view(b, h, w, nH, hdp)[..., hd:].abs().max().item() == 0
    dop = F.pad(dout.view(b, h, w, nH, hd), (0, hdp - hd)).reshape(b, h, w, nH * hdp).to(cuda).contiguous()
    dqkv, dtab = S.window_attn_bwd(qp, out, dop, lse, g, b, h, w, scale, table.to(cuda))
    dq = dqkv.view(b, h, w, 3, nH, hdp)[..., :hd].reshape(b, h, w, 3 * C).double().cpu()
    gref = qd.grad
    assert (dq - gref).abs().max().item() < tol * max(1.0, gref.abs().max().item())
    assert (dtab.double().cpu() - td.grad).abs().max().item() < tol * max(1.0, td.grad.abs().max().item())


@pytest.mark.parametrize('shift', [0, 4])
@pytest.mark.parametrize('geom', [(2, 16, 24, 6, 30), (3, 8, 40, 3, 32), (1, 24, 24, 2, 16), (32, 8, 8, 6, 30)])
def test_window_attention_bwd_reduce_paths_bitwise(cuda, shift, geom):
    """The MFMA backward's table gradient (per-lane slot rows folded in a fixed order by
    wattn_dbias_slots / _fold, round 5: quarter sums + one wave per (head, bin)): the fused reduce and
    the deferred one (sr_window_attn_dbias_reduce, the side-stream path) are bitwise equal, a repeat run
    is bitwise equal (deterministic), and both match the fp64 oracle (window counts not a multiple of
    the 4 windows per wave included; B 32 at one window per image: many slot rows per head)."""
    b, h, w, nH, hd = geom
    torch.manual_seed(7)
    C = nH * hd
    g = S.AttnGeom(C, nH, 8, shift if min(h, w) > 8 else 0, 32)
    sh = g.shift
    qkv_raw = torch.randn(b, h, w, 3 * C).to(torch.bfloat16)
    qkv = _qkv_padded(qkv_raw, nH, hd, 32).to(cuda).contiguous()
    table = (torch.randn(225, nH) * 0.5)
    dout_raw = torch.randn(b, h, w, nH, hd).to(torch.bfloat16)
    dout = F.pad(dout_raw, (0, 32 - hd)).reshape(b, h, w, nH * 32).to(cuda).contiguous()
    scale = hd**-0.5
    out, lse = S.window_attn(qkv, g, b, h, w, scale, table.to(cuda))
    res = [S.window_attn_bwd(qkv, out, dout, lse, g, b, h, w, scale, table.to(cuda)) for _ in range(2)]
    torch.cuda.synchronize()
    from basicsr4rs_amd import _lib
    lib = _lib.load()
    wsb = lib.sr_window_attn_bwd_workspace(b, h, w, 8, nH)
    ws = torch.empty(wsb // 4 + 1, device=cuda, dtype=torch.float32)
    dq2, dt2 = torch.empty_like(qkv), torch.zeros(225, nH, device=cuda)
    _lib.check(lib.sr_window_attn_bwd(_lib.dtype_code(qkv.dtype), _lib.ptr(qkv), qkv.shape[-1], _lib.ptr(out),
                                      _lib.ptr(dout), out.shape[-1], _lib.ptr(lse), b, h, w, 8, sh, nH, hd, 32,
                                      float(scale), _lib.ptr(table.to(cuda)), _lib.ptr(dq2), _lib.ptr(dt2), _lib.ptr(ws),
                                      wsb, 2, _lib.stream()))
    parts = lib.sr_window_attn_bwd_parts(_lib.dtype_code(qkv.dtype), b, h, w, 8, nH, hd, 32, qkv.shape[-1],
                                         out.shape[-1])
    assert parts < 0  # slot rows
    _lib.check(lib.sr_window_attn_dbias_reduce(_lib.ptr(ws), parts, nH, 8, _lib.ptr(dt2), 1, _lib.stream()))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert torch.equal(dq2, res[0][0]) and torch.equal(dt2, res[0][1])
    qd = qkv_raw.double().requires_grad_()
    td = table.double().requires_grad_()
    ref = O.window_attention_core(qd, nH, 8, sh, scale, td)
    ref.backward(dout_raw.reshape(b, h, w, C).double())
    assert (res[0][1].double().cpu() - td.grad).abs().max().item() < 2e-2 * max(1.0, td.grad.abs().max().item())


@pytest.mark.parametrize('which', ['qkv', 'fc1'])
@pytest.mark.parametrize('shape', [(2, 16, 16, 180, 6), (1, 8, 24, 60, 6), (3, 5, 13, 96, 3)])
def test_linear_ln_fused_vs_separate(cuda, which, shape):
    """sr_linear_ln_fwd (LayerNorm in the lin kernel's prologue) against the standalone LayerNorm
    kernel followed by the linear: the normalised rows, mean / rstd, the GELU' side output (against
    float64 GELU' of the pre-activation) and the output; ragged last token tile (M % 128 != 0) included."""
    from basicsr4rs_amd.ops import swin as S
    N, H, W, C_, nH = shape
    torch.manual_seed(3)
    dt = torch.bfloat16
    Cp = (C_ + 7) // 8 * 8
    x = torch.zeros(N, H, W, Cp, device=cuda)
    x[..., :C_] = torch.randn(N, H, W, C_, device=cuda) * 2 + 0.5
    x = x.to(dt)
    g = torch.nn.Parameter(torch.rand(C_, device=cuda) + 0.5)
    b = torch.nn.Parameter(torch.randn(C_, device=cuda) * 0.1)
    if which == 'qkv':
        spec = S.qkv_spec(C_, nH, 32)
        lin = torch.nn.Linear(C_, 3 * C_).to(cuda)
        act, aux = 0, None
    else:
        spec = S.plain_spec(C_, 2 * C_)
        lin = torch.nn.Linear(C_, 2 * C_).to(cuda)
        act = S.GELU
        aux = torch.empty(N, H, W, spec.cout_p, device=cuda, dtype=dt)
    wf, _, bg = S.prepared_linear(lin.weight, lin.bias, spec, dt)
    y, ln, mean, rstd = S.linear_ln_fwd(x, g, b, C_, wf, bg, spec, N, H, W, act=act, aux=aux)
    ln_r, mean_r, rstd_r = S.layernorm(x, g, b, C_)
    aux_r = torch.empty_like(aux) if aux is not None else None
    y_r = S.linear_fwd(ln_r, wf, bg, spec, N, H, W, act=act, aux=aux_r)
    torch.cuda.synchronize()
    assert (mean - mean_r).abs().max().item() <= 1e-5 * max(1.0, mean_r.abs().max().item())
    assert (rstd - rstd_r).abs().max().item() <= 1e-4 * rstd_r.abs().max().item()
    assert (ln.float() - ln_r.float()).abs().max().item() <= 2e-2 * ln_r.float().abs().max().item()
    assert torch.equal(ln[..., C_:], torch.zeros_like(ln[..., C_:]))
    assert (y.float() - y_r.float()).abs().max().item() <= 2e-2 * max(1.0, y_r.float().abs().max().item())
    if aux is not None:
        assert (aux.float() - aux_r.float()).abs().max().item() <= 2e-2 * max(1.0, aux_r.float().abs().max().item())
        # the aux of a GELU linear is GELU' of the pre-activation (the fc2 dgrad's gate multiplies by it)
        pre = ln_r[..., :C_].double() @ lin.weight.detach().to(dt).double().t() + lin.bias.detach().double()
        dref = 0.5 * (1 + torch.erf(pre / 2**0.5)) + pre * torch.exp(-pre * pre / 2) / (2 * torch.pi) ** 0.5
        got = aux[..., :2 * C_].double()
        assert (got - dref).abs().max().item() <= 2e-2, (got - dref).abs().max().item()


@pytest.mark.parametrize('K,Cout', [(360, 184), (576, 184), (200, 96), (256, 304), (384, 40), (184, 184), (184, 360)])
@pytest.mark.parametrize('epi', ['plain', 'res', 'res_rowscale', 'gate'])
def test_linear_wide_k_vs_fp64(cuda, K, Cout, epi):
    """Wide-K linears (192 < K <= 576: SwinIR fc2 fwd 360 -> 184, fc1 / qkv dgrads 360 / 576 -> 184) --
    linear_wk_kernel for 96 < Cout <= 384, the 64-token lin kernel otherwise (and with variant 64) --
    against float64 on the same bf16 operands, with the epilogues those calls use (residual, residual
    + per-image row scale, GELU' gate) and a ragged last token tile; variant 55 (the 256x256 pp kernel
    for these shapes) agrees within bf16 rounding."""
    from basicsr4rs_amd import _lib
    from basicsr4rs_amd.ops import conv as C
    # 960 tokens (ragged against 128- and 64-token tiles); the row scale needs H*W % 128 == 0
    N, H, W = (3, 8, 48) if epi == 'res_rowscale' else (3, 8, 40)
    torch.manual_seed(K + Cout)
    dt = torch.bfloat16
    x = (torch.randn(N, H, W, K, device=cuda) * 0.5).to(dt)
    w = (torch.randn(Cout, K, device=cuda) * K**-0.5)
    bias = torch.randn(Cout, device=cuda) * 0.1
    wf = w.to(dt).contiguous()
    res = (torch.randn(N, H, W, Cout, device=cuda)).to(dt) if epi.startswith('res') else None
    gate = (torch.randn(N, H, W, Cout, device=cuda)).to(dt) if epi == 'gate' else None
    rs = (torch.rand(N, device=cuda) + 0.5) if epi == 'res_rowscale' else None
    kw = {}
    if res is not None:
        kw.update(res=res, beta=1.0)
    if rs is not None:
        kw.update(row_scale=rs)
    if gate is not None:
        kw.update(gate=gate, gate_mode=1)  # times the stored GELU' map g (the fc2 dgrad gate)

    def run():
        y = torch.empty(N, H, W, Cout, device=cuda, dtype=dt)
        C.conv_fwd_raw(x, wf, bias, y, N, H, W, K, Cout, Cout, ksize=1, **kw)
        return y

    lib = _lib.load()
    d = C._desc(dt, N, H, W, K, K, Cout, Cout, Cout, ksize=1)
    assert lib.sr_conv3x3_fwd_kernel_name(d) == (b'linear_wk_kernel' if 96 < Cout <= 384 else b'conv3x3_lin_kernel')
    y = run().double()
    ref = x.double() @ w.to(dt).double().t() + bias.double()
    if gate is not None:
        gd = gate.double()
        ref = ref * gd
    if rs is not None:
        ref = ref * rs.double().view(N, 1, 1, 1)
    if res is not None:
        ref = ref + res.double()
    tol = 1e-2 * max(1.0, ref.abs().max().item())
    assert (y - ref).abs().max().item() <= tol
    _lib.check(lib.sr_conv3x3_set_variant(55))
    try:
        assert lib.sr_conv3x3_fwd_kernel_name(d) != b'conv3x3_lin_kernel' or K <= 192
        y55 = run().double()
        _lib.check(lib.sr_conv3x3_set_variant(64))
        assert lib.sr_conv3x3_fwd_kernel_name(d) == b'conv3x3_lin_kernel'
        y64 = run().double()
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    assert (y55 - ref).abs().max().item() <= tol
    assert (y64 - ref).abs().max().item() <= tol
