"""Fused residual blocks of RCAN and RRDBNet, and the MSRResNet bilinear skip, on the HIP engine.

Each block is one autograd Function whose forward/backward are sequences of libsr_hip
launches (implicit-GEMM convs with fused epilogues + the HBM kernels of csrc/blocks.hip):

* ``rcab``  — RCAB (basicsr/archs/rcan_arch.py:27-46): conv-ReLU-conv, ChannelAttention
  (avg-pool, 1x1 C->C/r, ReLU, 1x1 C/r->C, sigmoid, rcan_arch.py:8-24), ``* res_scale + x``.
* ``rrdb``  — RRDB of three ResidualDenseBlocks (rrdbnet_arch.py:9-63): the dense concats are
  channel slices of one [N, H, W, nf + 4*gc] buffer per RDB (convs read/write slices in place,
  no torch.cat copies); the two residual scalings of the last RDB fuse into its conv5 epilogue.
* ``bilinear_up_add`` — MSRResNet ``out += F.interpolate(x, bilinear)`` (srresnet_arch.py:64-65).
"""

import torch

from .. import _lib
from . import conv as C
from .._switches import switch


# SR_CA_UNFUSED=1: the round-2 channel-attention launches (A/B of the fused kernels, tools/ab_env.sh)
_CA_UNFUSED = switch('SR_CA_UNFUSED') == '1'


def _ws(nbytes, device):
    return torch.empty(max(1, nbytes // 4 + 1), device=device, dtype=torch.float32)


def channel_reduce(a, b=None, scale=1.0, C_=None, coff=0):
    """out[n, c] = scale * sum_p a[n, p, c] (* b) for NHWC a (fp32 result)."""
    N, H, W, ld = a.shape
    Cc = C_ or ld
    lib = _lib.load()
    wsb = lib.sr_channel_reduce_workspace(N, H * W, Cc)
    ws = _ws(wsb, a.device)
    out = torch.empty(N, Cc, device=a.device, dtype=torch.float32)
    _lib.check(
        lib.sr_channel_reduce(_lib.dtype_code(a.dtype), _lib.ptr(a), ld, coff, _lib.ptr(b), b.shape[-1] if b is not None
                              else 0, coff, N, H * W, Cc, float(scale), _lib.ptr(out), _lib.ptr(ws), wsb,
                              _lib.stream()))
    return out


def nc_affine(x, u, s, t, beta, alpha, gamma):
    N, H, W, Cc = u.shape
    out = torch.empty_like(u)
    lib = _lib.load()
    _lib.check(
        lib.sr_nc_affine(_lib.dtype_code(u.dtype), _lib.ptr(x), _lib.ptr(u), _lib.ptr(s), _lib.ptr(t), N, H * W, Cc,
                         float(beta), float(alpha), float(gamma), _lib.ptr(out), _lib.stream()))
    return out


def _colsum_ok(N, H, W, spec, dtype):
    d = C._desc(dtype, N, H, W, spec.cin_p, spec.cin_p, spec.cout_p, spec.cout, spec.cout_p)
    return _lib.load().sr_conv3x3_fwd_colsum_parts(d) > 0


# SR_CA_DOT=1 (opt-in): the channel-attention dot partials dy * u from the next block's conv1 dgrad
# epilogue (the band kernel's dot epilogue) instead of their own pass (sr_channel_partials).  Measured
# slower every round: rounds 3-5 blamed the band kernel's 128 partial rows per image, which ca_bwd_apply
# stages per block; round 6 sums them per band (16 rows per image at B 32, the pass's own count) and it
# is still slower (RCAN x4 35.15 / 35.15 vs 33.49 / 33.35 ms, profiles/r06/ab/cadot/): the dot form of
# the dgrad runs 30.2 vs 20.1 us (residual only), more than the 8.9 us pass it replaces.
_CA_DOT_FUSED = switch('SR_CA_DOT') == '1'


def _dot_parts_put(dx, parts, u):
    """Attach the partial dots of dx * u (the previous RCAB's conv2 output) to dx, with dx's version
    counter: autograd hands dx to that block's backward as its dy."""
    dx._sr_ca_dot = (parts, u.data_ptr(), dx._version)


def _dot_parts_take(dy, u):
    """The fused partial dots of dy * u if dy carries them for this u and was not modified since (an
    in-place gradient accumulation bumps the version); else None."""
    e = getattr(dy, '_sr_ca_dot', None)
    if e is None:
        return None
    dy._sr_ca_dot = None
    parts, uptr, ver = e
    return parts if (uptr == u.data_ptr() and dy._version == ver) else None


class _RCAB(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, aw1, ab1, aw2, ab2, spec1, spec2, rs):
        dtype = x.dtype
        N, H, W, Cp = x.shape
        # x is the previous RCAB's output: its conv2 output u rides on it (_sr_ca_u), and this block's
        # conv1 dgrad -- which produces that block's dy -- also emits the partial dots dy * u its
        # channel-attention backward needs (the band kernel's dot epilogue, _dot_parts_put / _take)
        u_prev = getattr(x, '_sr_ca_u', None) if _CA_DOT_FUSED else None
        ctx.u_prev = u_prev if (u_prev is not None and u_prev.shape == x.shape and u_prev.dtype == dtype and
                                C.dot_partials_ok(dtype, N, H, W, spec1.cout_p, spec1.cin_p)) else None
        wf1, _, bg1 = C.prepared(w1, b1, spec1, dtype)
        wf2, _, bg2 = C.prepared(w2, b2, spec2, dtype)
        t = torch.empty(N, H, W, spec1.cout_p, device=x.device, dtype=dtype)
        C.conv_fwd_raw(x, wf1, bg1, t, N, H, W, spec1.cin_p, spec1.cout_p, spec1.cout, act=_lib.ACT_RELU)
        u = torch.empty(N, H, W, spec2.cout_p, device=x.device, dtype=dtype)
        lib = _lib.load()
        # AdaptiveAvgPool2d(1) of u: per-wave channel partial sums from conv2's epilogue (when the
        # conv kernel provides them), summed inside the squeeze-MLP kernel
        cs = _colsum_ok(N, H, W, spec2, dtype)
        r = C.conv_fwd_raw(t, wf2, bg2, u, N, H, W, spec2.cin_p, spec2.cout_p, spec2.cout, colsum=cs)
        if cs:
            parts = r[1]
        else:
            parts = torch.empty(N, lib.sr_channel_partials_count(H * W), Cp, device=x.device, dtype=torch.float32)
            _lib.check(lib.sr_channel_partials(_lib.dtype_code(dtype), _lib.ptr(u), Cp, 0, None, 0, 0, N, H * W, Cp,
                                               _lib.ptr(parts), _lib.stream()))
        Cr = aw1.shape[0]
        a1 = aw1.detach().reshape(Cr, -1)
        a2 = aw2.detach().reshape(-1, Cr)
        pool = torch.empty(N, Cp, device=x.device, dtype=torch.float32)
        h = torch.empty(N, Cr, device=x.device, dtype=torch.float32)
        s = torch.empty(N, Cp, device=x.device, dtype=torch.float32)
        # the fused kernels stage the partial rows and squeeze weights in LDS (csrc/blocks.hip limits)
        fused = (not _CA_UNFUSED and parts.shape[1] * Cp <= 8192 and Cp * Cr <= 2048 and Cp <= 256 and Cr <= 64
                 and N * Cp <= 4096 and N * Cr <= 1024)
        ctx.ca_fused = fused
        if not fused:  # the separate squeeze-MLP launch + elementwise pass (A/B, or shapes past the limits)
            _lib.check(
                lib.sr_ca_mlp_fwd(_lib.ptr(parts), parts.shape[1], 1.0 / (H * W), _lib.ptr(a1),
                                  _lib.ptr(ab1.detach() if ab1 is not None else None), _lib.ptr(a2),
                                  _lib.ptr(ab2.detach() if ab2 is not None else None), N, Cp, Cr, _lib.ptr(pool),
                                  _lib.ptr(h), _lib.ptr(s), _lib.stream()))
            y = nc_affine(x, u, s, None, 1.0, rs, 0.0)
            ctx.specs = (spec1, spec2)
            ctx.rs = rs
            ctx.save_for_backward(x, t, u, pool, h, s, w1, b1, w2, b2, aw1, aw2, ab1, ab2)
            y._sr_ca_u = u
            return y
        y = torch.empty_like(u)
        # squeeze MLP + y = x + rs * u * s in one launch (csrc/blocks.hip ca_fwd_apply_kernel)
        _lib.check(
            lib.sr_ca_fwd_apply(_lib.dtype_code(dtype), _lib.ptr(parts), parts.shape[1], 1.0 / (H * W), _lib.ptr(a1),
                                _lib.ptr(ab1.detach() if ab1 is not None else None), _lib.ptr(a2),
                                _lib.ptr(ab2.detach() if ab2 is not None else None), _lib.ptr(x), _lib.ptr(u), N,
                                H * W, Cp, Cr, float(rs), _lib.ptr(y), _lib.ptr(pool), _lib.ptr(h), _lib.ptr(s),
                                _lib.stream()))
        ctx.specs = (spec1, spec2)
        ctx.rs = rs
        ctx.save_for_backward(x, t, u, pool, h, s, w1, b1, w2, b2, aw1, aw2, ab1, ab2)
        y._sr_ca_u = u
        return y

    @staticmethod
    def backward(ctx, dy):
        # the block's three side-stream launches (squeeze-conv gradients, both conv weight
        # gradients) forked once, after conv1's dgrad (ops.conv.side_batch)
        with C.side_batch():
            return _RCAB._backward_body(ctx, dy)

    @staticmethod
    def _backward_body(ctx, dy):
        x, t, u, pool, h, s, w1, b1, w2, b2, aw1, aw2, ab1, ab2 = ctx.saved_tensors
        spec1, spec2 = ctx.specs
        rs = ctx.rs
        dtype = x.dtype
        N, H, W, Cp = x.shape
        Cr = aw1.shape[0]
        a1 = aw1.detach().reshape(Cr, -1)
        a2 = aw2.detach().reshape(-1, Cr)
        parts = _dot_parts_take(dy, u)  # emitted by the next block's conv1 dgrad, which produced dy
        dy = dy.to(dtype).contiguous()
        lib = _lib.load()
        if parts is None:
            # dL/ds[n,c] = rs * sum_p dy*u: per-chunk dot partials, summed in the MLP backward kernel
            parts = torch.empty(N, lib.sr_channel_partials_count(H * W), Cp, device=x.device, dtype=torch.float32)
            _lib.check(lib.sr_channel_partials(_lib.dtype_code(dtype), _lib.ptr(dy), Cp, 0, _lib.ptr(u), Cp, 0, N,
                                               H * W, Cp, _lib.ptr(parts), _lib.stream()))
        if not ctx.ca_fused or parts.shape[1] * Cp > 8192:
            return _RCAB._backward_unfused(ctx, dy, parts, x, t, u, pool, h, s, w1, b1, w2, b2, aw1, aw2, ab1, ab2,
                                           spec1, spec2, rs, a1, a2, Cr, N, H, W, Cp, dtype)
        # squeeze-MLP backward + du = rs * dy * s + dpool / HW in one launch; the squeeze convs'
        # parameter gradients follow from the per-image dz2 / dz1 in their own small launch, on
        # the weight-gradient side stream when one is active (they only feed the optimizer)
        du = torch.empty_like(dy)
        dz2 = torch.empty(N, Cp, device=x.device, dtype=torch.float32)
        dz1 = torch.empty(N, Cr, device=x.device, dtype=torch.float32)
        _lib.check(
            lib.sr_ca_bwd_apply(_lib.dtype_code(dtype), _lib.ptr(parts), parts.shape[1], float(rs), _lib.ptr(s),
                                _lib.ptr(h), _lib.ptr(a1), _lib.ptr(a2), _lib.ptr(dy), N, H * W, Cp, Cr, _lib.ptr(du),
                                _lib.ptr(dz2), _lib.ptr(dz1), _lib.stream()))
        # squeeze-conv gradients: straight into the optimizer's flat .grad views when they exist
        ca = (aw1, ab1, aw2, ab2)
        tg = [C.grad_target(p) for p in ca]
        direct = all(g is not None for g in tg)
        if direct:
            dA1, dab1, dA2, dab2 = tg
        else:
            dA1, dA2 = torch.empty_like(a1), torch.empty_like(a2)
            dab1 = torch.empty(Cr, device=x.device, dtype=torch.float32) if ab1 is not None else None
            dab2 = torch.empty(Cp, device=x.device, dtype=torch.float32) if ab2 is not None else None
        args = (_lib.ptr(dz2), _lib.ptr(dz1), _lib.ptr(h), _lib.ptr(pool), N, Cp, Cr, _lib.ptr(dA1), _lib.ptr(dab1),
                _lib.ptr(dA2), _lib.ptr(dab2), int(direct))
        side = C.async_side_stream(x.device) if direct else None
        if side is not None:
            C.side_launch(side, lambda: _lib.check(lib.sr_ca_param_grad(*args, _lib.stream())), (dz2, dz1, h, pool),
                          after=tuple((lambda p=p: C.grad_ready(p)) for p in ca))
        else:
            _lib.check(lib.sr_ca_param_grad(*args, _lib.stream()))
            if direct:
                for p in ca:
                    C.grad_ready(p)
        _, wd1, _ = C.prepared(w1, b1, spec1, dtype)
        _, wd2, _ = C.prepared(w2, b2, spec2, dtype)
        dz1 = torch.empty_like(t)
        C.conv_fwd_raw(du, wd2, None, dz1, N, H, W, spec2.cout_p, spec2.cin_p, spec2.cin_p, gate=t, gate_slope=0.0)
        dw2, db2 = C.conv_wgrad_raw(du, t, N, H, W, spec2.cin_p, spec2.cin, spec2.cout_p, spec2.cout, params=(w2, b2))
        dx = torch.empty_like(x)
        if ctx.u_prev is not None:  # dx is the previous block's dy: its CA dot partials in the same pass
            _, dparts = C.conv_fwd_raw(dz1, wd1, None, dx, N, H, W, spec1.cout_p, spec1.cin_p, spec1.cin_p, res=dy,
                                       beta=1.0, colsum=True, dot=ctx.u_prev)
            _dot_parts_put(dx, dparts, ctx.u_prev)
        else:
            C.conv_fwd_raw(dz1, wd1, None, dx, N, H, W, spec1.cout_p, spec1.cin_p, spec1.cin_p, res=dy, beta=1.0)
        dw1, db1 = C.conv_wgrad_raw(dz1, x, N, H, W, spec1.cin_p, spec1.cin, spec1.cout_p, spec1.cout, params=(w1, b1))
        if direct:
            return dx, dw1, db1, dw2, db2, None, None, None, None, None, None, None
        return (dx, dw1, db1, dw2, db2, dA1.reshape(Cr, Cp, 1, 1), dab1, dA2.reshape(Cp, Cr, 1, 1), dab2, None, None,
                None)


def _rcab_backward_unfused(ctx, dy, parts, x, t, u, pool, h, s, w1, b1, w2, b2, aw1, aw2, ab1, ab2, spec1, spec2, rs,
                           a1, a2, Cr, N, H, W, Cp, dtype):
    """The round-2 RCAB backward (single-block squeeze-MLP backward, then the du pass): A/B only."""
    lib = _lib.load()
    dpool = torch.empty(N, Cp, device=x.device, dtype=torch.float32)
    ca = (aw1, ab1, aw2, ab2)
    tg = [C.grad_target(p) for p in ca]
    direct = all(g is not None for g in tg)
    if direct:
        dA1, dab1, dA2, dab2 = tg
    else:
        dA1, dA2 = torch.empty_like(a1), torch.empty_like(a2)
        dab1 = torch.empty(Cr, device=x.device, dtype=torch.float32) if ab1 is not None else None
        dab2 = torch.empty(Cp, device=x.device, dtype=torch.float32) if ab2 is not None else None
    _lib.check(
        lib.sr_ca_mlp_bwd(_lib.ptr(parts), parts.shape[1], rs, _lib.ptr(s), _lib.ptr(h), _lib.ptr(pool), _lib.ptr(a1),
                          _lib.ptr(a2), N, Cp, Cr, _lib.ptr(dpool), _lib.ptr(dA1), _lib.ptr(dab1), _lib.ptr(dA2),
                          _lib.ptr(dab2), int(direct), _lib.stream()))
    if direct:
        for p in ca:
            C.grad_ready(p)
    du = nc_affine(None, dy, s, dpool, 0.0, rs, 1.0 / (H * W))
    _, wd1, _ = C.prepared(w1, b1, spec1, dtype)
    _, wd2, _ = C.prepared(w2, b2, spec2, dtype)
    dz1 = torch.empty_like(t)
    C.conv_fwd_raw(du, wd2, None, dz1, N, H, W, spec2.cout_p, spec2.cin_p, spec2.cin_p, gate=t, gate_slope=0.0)
    dw2, db2 = C.conv_wgrad_raw(du, t, N, H, W, spec2.cin_p, spec2.cin, spec2.cout_p, spec2.cout, params=(w2, b2))
    dx = torch.empty_like(x)
    C.conv_fwd_raw(dz1, wd1, None, dx, N, H, W, spec1.cout_p, spec1.cin_p, spec1.cin_p, res=dy, beta=1.0)
    dw1, db1 = C.conv_wgrad_raw(dz1, x, N, H, W, spec1.cin_p, spec1.cin, spec1.cout_p, spec1.cout, params=(w1, b1))
    if direct:
        return dx, dw1, db1, dw2, db2, None, None, None, None, None, None, None
    return (dx, dw1, db1, dw2, db2, dA1.reshape(Cr, Cp, 1, 1), dab1, dA2.reshape(Cp, Cr, 1, 1), dab2, None, None, None)


_RCAB._backward_unfused = staticmethod(_rcab_backward_unfused)


def rcab(x, conv1, conv2, ca1, ca2, res_scale):
    """RCAB on an NHWC map; conv1/conv2 3x3 nn.Conv2d, ca1/ca2 the 1x1 squeeze convs."""
    if C.pad8(conv1.in_channels) != conv1.in_channels:
        raise ValueError('RCAB needs num_feat divisible by 8')
    s1 = C.ConvSpec(conv1.in_channels, conv1.out_channels, act=_lib.ACT_RELU)
    s2 = C.ConvSpec(conv2.in_channels, conv2.out_channels)
    return _RCAB.apply(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, ca1.weight, ca1.bias, ca2.weight,
                       ca2.bias, s1, s2, float(res_scale))


def _copy_channels(src, lds_, scoff, dst, ldd, dcoff, P, Cc):
    lib = _lib.load()
    _lib.check(lib.sr_copy_channels(_lib.dtype_code(src.dtype), _lib.ptr(src), lds_, scoff, _lib.ptr(dst), ldd, dcoff,
                                    P, Cc, _lib.stream()))


def _act_bwd_inplace(buf, yb, Cbuf, coff, Cc, P, slope):
    lib = _lib.load()
    _lib.check(
        lib.sr_act_backward_nhwc(_lib.dtype_code(buf.dtype), P, Cc, _lib.ptr(buf), Cbuf, coff, _lib.ptr(yb), Cbuf, coff,
                                 _lib.ptr(buf), Cbuf, coff, _lib.ACT_LRELU, float(slope), 1.0, _lib.stream()))


class _RRDB(torch.autograd.Function):
    """RRDB: out = 0.2 * rdb3(rdb2(rdb1(x))) + x, RDB(z) = 0.2 * conv5(cat(z, x1..x4)) + z."""

    @staticmethod
    def forward(ctx, x, nf, gc, *params):
        dtype = x.dtype
        N, H, W, _ = x.shape
        Cb = nf + 4 * gc
        P = N * H * W
        specs = [C.ConvSpec(nf + k * gc, gc if k < 4 else nf) for k in range(5)]
        bufs = [torch.empty(N, H, W, Cb, device=x.device, dtype=dtype)]
        _copy_channels(x, nf, 0, bufs[0], Cb, 0, P, nf)
        out = None
        for r in range(3):
            B = bufs[r]
            for k in range(4):  # x_{k+1} = lrelu(conv_{k+1}(B[0 : nf + k*gc])) -> B[nf + k*gc : +gc]
                wf, _, bg = C.prepared(params[r * 10 + 2 * k], params[r * 10 + 2 * k + 1], specs[k], dtype)
                C.conv_fwd_raw(B, wf, bg, B, N, H, W, nf + k * gc, gc, gc, act=_lib.ACT_LRELU, slope=0.2, ldx=Cb,
                               ldy=Cb, ycoff=nf + k * gc)
            wf5, _, bg5 = C.prepared(params[r * 10 + 8], params[r * 10 + 9], specs[4], dtype)
            if r < 2:  # next RDB input = 0.2 * conv5 + z, written into the next buffer's slice 0..nf
                nxt = torch.empty(N, H, W, Cb, device=x.device, dtype=dtype)
                C.conv_fwd_raw(B, wf5, bg5, nxt, N, H, W, Cb, nf, nf, res=B, alpha=0.2, beta=1.0, ldx=Cb, ldy=Cb,
                               ldr=Cb)
                bufs.append(nxt)
            else:  # RRDB output = 0.2 * (0.2 * conv5 + z) + x
                out = torch.empty(N, H, W, nf, device=x.device, dtype=dtype)
                C.conv_fwd_raw(B, wf5, bg5, out, N, H, W, Cb, nf, nf, res=B, alpha=0.04, beta=0.2, res2=x, beta2=1.0,
                               ldx=Cb, ldy=nf, ldr=Cb, ldr2=nf)
        ctx.nf, ctx.gc = nf, gc
        ctx.specs = specs
        ctx.save_for_backward(x, *bufs, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        with C.side_batch():  # with side-stream weight gradients: one fork per RRDB (ops.conv.side_batch)
            return _RRDB._backward_body(ctx, dout)

    @staticmethod
    def _backward_body(ctx, dout):
        saved = ctx.saved_tensors
        x, bufs, params = saved[0], saved[1:4], saved[4:]
        nf, gc, specs = ctx.nf, ctx.gc, ctx.specs
        dtype = x.dtype
        N, H, W, _ = x.shape
        Cb = nf + 4 * gc
        P = N * H * W
        dout = dout.to(dtype).contiguous()
        grads = [None] * len(params)
        d_in = dout  # gradient of the current RDB's output, [N,H,W,nf] or slice 0..nf of a Cb buffer
        ld_in = nf
        for r in (2, 1, 0):
            B = bufs[r]
            w5, b5 = params[r * 10 + 8], params[r * 10 + 9]
            _, wd5, _ = C.prepared(w5, b5, specs[4], dtype)
            dB = torch.empty(N, H, W, Cb, device=x.device, dtype=dtype)
            a5 = 0.04 if r == 2 else 0.2
            rb = 0.2 if r == 2 else 1.0
            # dB[0:Cb] = a5 * dgrad5(d_in) ; dB[0:nf] += rb * d_in  (RDB skip); slice 3 (x4) is complete
            # here, so its LeakyReLU backward is applied in the same epilogue (post-residual gate)
            C.conv_fwd_raw(d_in, wd5, None, dB, N, H, W, nf, Cb, Cb, alpha=a5, res=d_in, beta=rb, rcols=nf, ldx=ld_in,
                           ldr=ld_in, ldy=Cb, gate=B, gate_slope=0.2, gate_mode=2, gcol0=nf + 3 * gc, gcol1=Cb)
            grads[r * 10 + 8], grads[r * 10 + 9] = C.conv_wgrad_raw(d_in, B, N, H, W, Cb, Cb, nf, nf, scale=a5,
                                                                   ldy=ld_in, ldx=Cb, params=(w5, b5))
            for k in (3, 2, 1, 0):
                co = nf + k * gc  # slice k (x_{k+1}) arrived complete and activation-backward'ed
                w, b = params[r * 10 + 2 * k], params[r * 10 + 2 * k + 1]
                _, wd, _ = C.prepared(w, b, specs[k], dtype)
                last = (r == 0 and k == 0)
                if last:
                    # d x = dB[0:nf] + dgrad1(dz1) + dout (RRDB skip) -> fresh [N,H,W,nf]
                    dx = torch.empty(N, H, W, nf, device=x.device, dtype=dtype)
                    C.conv_fwd_raw(dB, wd, None, dx, N, H, W, gc, co, co, res=dB, beta=1.0, res2=dout, beta2=1.0,
                                   ldx=Cb, xcoff=co, ldr=Cb, ldr2=nf, ldy=nf)
                elif k > 0:
                    # dB[0:co] += dgrad_k; this completes slice k-1, whose LeakyReLU backward rides along
                    C.conv_fwd_raw(dB, wd, None, dB, N, H, W, gc, co, co, res=dB, beta=1.0, ldx=Cb, xcoff=co, ldr=Cb,
                                   ldy=Cb, gate=B, gate_slope=0.2, gate_mode=2, gcol0=co - gc, gcol1=co)
                else:  # k == 0: dB[0:nf] is the RDB input's gradient (no activation)
                    C.conv_fwd_raw(dB, wd, None, dB, N, H, W, gc, co, co, res=dB, beta=1.0, ldx=Cb, xcoff=co, ldr=Cb,
                                   ldy=Cb)
                grads[r * 10 + 2 * k], grads[r * 10 + 2 * k + 1] = C.conv_wgrad_raw(
                    dB, B, N, H, W, co, co, gc, gc, ldy=Cb, ycoff=co, ldx=Cb, params=(w, b))
            d_in, ld_in = dB, Cb
        return (dx, None, None, *grads)


def rrdb(x, block):
    """x: NHWC [N,H,W,nf]; block: an RRDB module (rdb1..3 with conv1..conv5)."""
    nf = block.rdb1.conv1.in_channels
    gc = block.rdb1.conv1.out_channels
    if nf % 8 or gc % 8:
        raise ValueError('RRDB on the HIP engine needs num_feat and num_grow_ch divisible by 8')
    params = []
    for rdb in (block.rdb1, block.rdb2, block.rdb3):
        for conv in (rdb.conv1, rdb.conv2, rdb.conv3, rdb.conv4, rdb.conv5):
            params += [conv.weight, conv.bias]
    return _RRDB.apply(x, nf, gc, *params)


class _BilinearAdd(torch.autograd.Function):

    @staticmethod
    def forward(ctx, out, x, s):
        N, Cc, H, W = x.shape
        y = torch.empty_like(out)
        lib = _lib.load()
        _lib.check(lib.sr_bilinear_up_add(_lib.ptr(x.contiguous().float()), N, Cc, H, W, int(s),
                                          _lib.ptr(out.contiguous()), _lib.ptr(y), _lib.stream()))
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.needs_input_grad[1]:
            raise NotImplementedError('gradient w.r.t. the LR input of the bilinear skip is not implemented')
        return dy, None, None


def bilinear_up_add(out, x, s):
    return _BilinearAdd.apply(out, x, s)
