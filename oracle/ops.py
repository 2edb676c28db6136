"""ORACLE — float64 numpy restatements of the basicsr/ops native extensions.

Test infrastructure only (tests/, __graft_entry__.smoke()); the product path never
imports it.  Each function restates the reference algorithm from its source:

* deformable conv v1/v2 — basicsr/ops/dcn/src/deform_conv_cuda_kernel.cu (bilinear
  sampling :85-116 / :468-498, im2col :191-250 / :571-634, col2im :280-372 / :636-694,
  col2im_coord :374-466 / :696-770) and the host GEMM composition of
  deform_conv_cuda.cpp:490-685;
* fused_bias_act — basicsr/ops/fused_act/src/fused_bias_act_kernel.cu (the act*10+grad
  switch);
* upfirdn2d — basicsr/ops/upfirdn2d/upfirdn2d.py:162-192 (upfirdn2d_native).

The reference ops need their CUDA extensions and cannot run here: these
restatements are pinned in tests/test_oracle_ops.py by independent formulations (torch
autograd of the forward for the DCN gradients, F.conv2d for upfirdn2d, the reference's
own output-size and gradient-padding formulas) — "parity unpinned" against the
reference binaries themselves.
"""
import numpy as np


# ----------------------------------------------------------------------------- DCN
def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _geometry(x, weight, stride, padding, dilation):
    N, C, H, W = x.shape
    _, _, kh, kw = weight.shape
    (sh, sw), (ph, pw), (dh, dw) = _pair(stride), _pair(padding), _pair(dilation)
    Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    return N, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, Ho, Wo


def _sample_points(offset, kh, kw, sh, sw, ph, pw, dh, dw, Ho, Wo, DG, coords='f32'):
    """Sampling coordinates [N, DG, K, Ho, Wo] (h, w): base grid + tap + offset
    (offset channel 2*tap = dy, 2*tap+1 = dx per deformable group, :604-615).

    coords='f32' rounds ``h_in + i*dil + offset`` to float32 exactly as the reference's
    fp32 kernel does (one rounding of int + float); the bilinear derivative is
    discontinuous at integer coordinates and at the -1 / H validity edges, so a sample
    within fp32 rounding of such a point must take the reference's branch.  'f64' keeps
    exact coordinates (used to pin the restatement against float64 autograd)."""
    N = offset.shape[0]
    K = kh * kw
    ft = np.float32 if coords == 'f32' else np.float64
    off = offset.reshape(N, DG, K, 2, Ho, Wo).astype(ft)
    ii, jj = np.divmod(np.arange(K), kw)
    hb = ((np.arange(Ho) * sh - ph)[None, :, None] + (ii * dh)[:, None, None]).astype(ft)  # [K, Ho, 1]
    wb = ((np.arange(Wo) * sw - pw)[None, None, :] + (jj * dw)[:, None, None]).astype(ft)  # [K, 1, Wo]
    h = (hb[None, None] + off[:, :, :, 0]).astype(np.float64)
    w = (wb[None, None] + off[:, :, :, 1]).astype(np.float64)
    return h, w


def _corners(h, w, H, W):
    """Corner indices / weights of the reference bilinear rule: valid iff h > -1, w > -1,
    h < H, w < W; corners outside the image contribute 0."""
    valid = (h > -1) & (w > -1) & (h < H) & (w < W)
    hl = np.floor(h).astype(np.int64)
    wl = np.floor(w).astype(np.int64)
    lh, lw = h - hl, w - wl
    hh, hw = 1 - lh, 1 - lw
    corners = []
    for dy, dx, wt in ((0, 0, hh * hw), (0, 1, hh * lw), (1, 0, lh * hw), (1, 1, lh * lw)):
        y, xx = hl + dy, wl + dx
        ok = valid & (y >= 0) & (y <= H - 1) & (xx >= 0) & (xx <= W - 1)
        corners.append((np.where(ok, y, 0), np.where(ok, xx, 0), ok, wt))
    return valid, (lh, lw, hh, hw), corners


def _gather(xc, y, xx, ok):
    """xc [N, Cg, H, W]; y/xx/ok [N, K, Ho, Wo] -> [N, Cg, K, Ho, Wo] (0 where not ok)."""
    n = np.arange(xc.shape[0])[:, None, None, None]
    v = xc[n, :, y, xx]  # [N, K, Ho, Wo, Cg]
    v = np.moveaxis(v, -1, 1)
    return np.where(ok[:, None], v, 0.0)


def dcn_columns(x, offset, mask, kh, kw, stride, padding, dilation, DG, coords='f32'):
    """cols[N, C, K, Ho, Wo] = mask * bilinear(x) (im2col, :571-634; mask None = v1)."""
    N, C, H, W = x.shape
    (sh, sw), (ph, pw), (dh, dw) = _pair(stride), _pair(padding), _pair(dilation)
    Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    K = kh * kw
    hs, ws = _sample_points(offset, kh, kw, sh, sw, ph, pw, dh, dw, Ho, Wo, DG, coords)
    m = np.ones((N, DG, K, Ho, Wo)) if mask is None else mask.reshape(N, DG, K, Ho, Wo).astype(np.float64)
    cpg = C // DG
    cols = np.zeros((N, C, K, Ho, Wo))
    x = x.astype(np.float64)
    for g in range(DG):
        xc = x[:, g * cpg:(g + 1) * cpg]
        valid, _, corners = _corners(hs[:, g], ws[:, g], H, W)
        val = 0.0
        for y, xx, ok, wt in corners:
            val = val + wt[:, None] * _gather(xc, y, xx, ok)
        cols[:, g * cpg:(g + 1) * cpg] = np.where(valid[:, None], val, 0.0) * m[:, g][:, None]
    return cols


def dcn_forward(x, offset, mask, weight, bias, stride, padding, dilation, groups, DG, coords='f32'):
    """out = per-group GEMM(weight.flatten(1), cols) + bias (deform_conv_cuda.cpp:490-557)."""
    N, C, H, W, kh, kw, *_, Ho, Wo = _geometry(x, weight, stride, padding, dilation)
    cols = dcn_columns(x, offset, mask, kh, kw, stride, padding, dilation, DG, coords)
    Cout = weight.shape[0]
    cg, og = C // groups, Cout // groups
    out = np.zeros((N, Cout, Ho, Wo))
    w = weight.astype(np.float64).reshape(Cout, cg, kh * kw)
    for g in range(groups):
        out[:, g * og:(g + 1) * og] = np.einsum('ock,nckhw->nohw', w[g * og:(g + 1) * og],
                                                cols[:, g * cg:(g + 1) * cg])
    if bias is not None:
        out += bias.astype(np.float64)[None, :, None, None]
    return out


def dcn_backward(x, offset, mask, weight, bias, stride, padding, dilation, groups, DG, dy, coords='f32'):
    """(grad_x, grad_offset, grad_mask, grad_weight, grad_bias), restating
    deform_conv_cuda.cpp:560-685: dcols = W^T dy per group; col2im_coord (offset, mask
    gradients from d bilinear / d h, d w), col2im (bilinear scatter of mask*dcols), and
    grad_weight = dy cols^T, grad_bias = sum dy."""
    N, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, Ho, Wo = _geometry(x, weight, stride, padding, dilation)
    K = kh * kw
    Cout = weight.shape[0]
    cg, og, cpg = C // groups, Cout // groups, C // DG
    x = x.astype(np.float64)
    dy = dy.astype(np.float64)
    w = weight.astype(np.float64).reshape(Cout, cg, K)
    dcols = np.zeros((N, C, K, Ho, Wo))
    for g in range(groups):
        dcols[:, g * cg:(g + 1) * cg] = np.einsum('ock,nohw->nckhw', w[g * og:(g + 1) * og], dy[:, g * og:(g + 1) * og])
    hs, ws = _sample_points(offset, kh, kw, sh, sw, ph, pw, dh, dw, Ho, Wo, DG, coords)
    m = np.ones((N, DG, K, Ho, Wo)) if mask is None else mask.reshape(N, DG, K, Ho, Wo).astype(np.float64)
    gx = np.zeros_like(x)
    goff = np.zeros((N, DG, K, 2, Ho, Wo))
    gmask = np.zeros((N, DG, K, Ho, Wo))
    nidx = np.broadcast_to(np.arange(N)[:, None, None, None], (N, K, Ho, Wo))
    for g in range(DG):
        sl = slice(g * cpg, (g + 1) * cpg)
        xc, dc = x[:, sl], dcols[:, sl]
        valid, (lh, lw, hh, hw), corners = _corners(hs[:, g], ws[:, g], H, W)
        vals = [_gather(xc, y, xx, ok) for y, xx, ok, _ in corners]  # v1..v4 [N, cpg, K, Ho, Wo]
        v1, v2, v3, v4 = vals
        dbil_h = -hw[:, None] * v1 - lw[:, None] * v2 + hw[:, None] * v3 + lw[:, None] * v4
        dbil_w = -hh[:, None] * v1 + hh[:, None] * v2 - lh[:, None] * v3 + lh[:, None] * v4
        bil = sum(wt[:, None] * v for (_, _, _, wt), v in zip(corners, vals))
        mg = m[:, g][:, None]
        vmask = valid[:, None]
        goff[:, g, :, 0] = np.where(vmask, dbil_h * dc * mg, 0.0).sum(1)
        goff[:, g, :, 1] = np.where(vmask, dbil_w * dc * mg, 0.0).sum(1)
        gmask[:, g] = np.where(vmask, dc * bil, 0.0).sum(1)
        t = np.where(vmask, dc * mg, 0.0)  # [N, cpg, K, Ho, Wo]
        for y, xx, ok, wt in corners:
            contrib = np.where(ok[:, None], wt[:, None] * t, 0.0)  # [N, cpg, K, Ho, Wo]
            for c in range(cpg):
                np.add.at(gx[:, g * cpg + c], (nidx, y, xx), contrib[:, c])
    cols = dcn_columns(x, offset, mask, kh, kw, stride, padding, dilation, DG, coords)
    gw = np.zeros((Cout, cg, K))
    for g in range(groups):
        gw[g * og:(g + 1) * og] = np.einsum('nohw,nckhw->ock', dy[:, g * og:(g + 1) * og], cols[:, g * cg:(g + 1) * cg])
    gb = dy.sum((0, 2, 3)) if bias is not None else None
    return (gx, goff.reshape(N, DG * K * 2, Ho, Wo), None if mask is None else gmask.reshape(N, DG * K, Ho, Wo),
            gw.reshape(weight.shape), gb)


# ----------------------------------------------------------------------- fused_act
def fused_bias_act(x, bias, ref, act, grad, alpha, scale):
    """fused_bias_act_kernel.cu: y = scale * f(x + b[(i // step_b) % size_b]) with
    f by act*10+grad (10/11 identity, 30 lrelu, 31 ref-gated slope, 12/32 zero)."""
    x = x.astype(np.float64)
    if bias is not None and bias.size:
        shape = [1] * x.ndim
        shape[1] = -1
        x = x + bias.astype(np.float64).reshape(shape)
    mode = act * 10 + grad
    if mode in (12, 32):
        y = np.zeros_like(x)
    elif mode == 30:
        y = np.where(x > 0, x, x * alpha)
    elif mode == 31:
        y = np.where(ref > 0, x, x * alpha)
    else:
        y = x
    return y * scale


def fused_lrelu_backward(dy, out, alpha, scale):
    """FusedLeakyReLUFunctionBackward.forward (fused_act.py:30-44): grad_input and the
    bias gradient (sum over every dim but 1)."""
    gi = fused_bias_act(dy, None, out, 3, 1, alpha, scale)
    dims = (0, ) + tuple(range(2, gi.ndim))
    return gi, gi.sum(dims)


# ----------------------------------------------------------------------- upfirdn2d
def upfirdn2d(x, kernel, up_x, up_y, down_x, down_y, px0, px1, py0, py1):
    """upfirdn2d_native (upfirdn2d.py:162-192) on [N, C, H, W]: zero-insert, pad / crop,
    correlate with the flipped kernel, subsample."""
    N, C, H, W = x.shape
    kh, kw = kernel.shape
    u = np.zeros((N, C, H * up_y, W * up_x))
    u[:, :, ::up_y, ::up_x] = x
    u = np.pad(u, ((0, 0), (0, 0), (max(py0, 0), max(py1, 0)), (max(px0, 0), max(px1, 0))))
    u = u[:, :, max(-py0, 0):u.shape[2] - max(-py1, 0), max(-px0, 0):u.shape[3] - max(-px1, 0)]
    kf = np.flip(kernel.astype(np.float64), (0, 1))
    Hf, Wf = u.shape[2] - kh + 1, u.shape[3] - kw + 1
    full = np.zeros((N, C, Hf, Wf))
    for i in range(kh):
        for j in range(kw):
            full += kf[i, j] * u[:, :, i:i + Hf, j:j + Wf]
    out_h = (H * up_y + py0 + py1 - kh) // down_y + 1
    out_w = (W * up_x + px0 + px1 - kw) // down_x + 1
    return full[:, :, ::down_y, ::down_x][:, :, :out_h, :out_w]
