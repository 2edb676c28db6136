"""C-ABI boundary checks that need no GPU: libsr_hip.so loads, exports every function
include/sr_hip.h declares, the ctypes signatures cover them, and argument validation
fails loudly with SR_EINVAL + a message (the reference raises RuntimeError from
TORCH_CHECK, basicsr/ops/dcn/src/deform_conv_cuda.cpp:511-516)."""
import ctypes
import os
import re

import pytest
import torch

from basicsr4rs_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, 'include', 'sr_hip.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(sr_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), f'{n} declared in include/sr_hip.h but not exported'
    assert set(names) == set(_lib.SIGNATURES), 'ctypes SIGNATURES out of sync with include/sr_hip.h'
    assert b'gfx950' in lib.sr_version()


def test_invalid_arguments_raise():
    lib = _lib.load()
    rc = lib.sr_conv3x3_fwd(None, None, None, None, None, None, None, None, None, None, None, None, None)
    assert rc == -1 and b'null' in lib.sr_last_error()
    with pytest.raises(RuntimeError, match='null'):
        _lib.check(rc)
    d = _lib.ConvDesc()
    d.dtype, d.N, d.H, d.W, d.Cin, d.ldx, d.Cout, d.ldw, d.ldy = 1, 1, 4, 4, 12, 12, 16, 108, 16
    dummy = ctypes.c_void_p(16)
    rc = lib.sr_conv3x3_fwd(d, dummy, dummy, None, None, None, None, None, None, dummy, None, None, None)
    assert rc == -1 and b'multiples of 8' in lib.sr_last_error()
    assert lib.sr_pixel_shuffle_nchw(0, dummy, 1, 3, 4, 4, 2, dummy, None) == -1  # C % r^2 != 0


def test_dcn_fused_forward_query_and_validation():
    """The fused DCN forward's shape query (host only) and its refusals (no launch)."""
    from basicsr4rs_amd.ops import dcn as D
    lib = _lib.load()

    def geom(C, Co, groups=1, dg=8):
        return D._Geom(torch.empty(2, C, 16, 16), torch.empty(Co, C // groups, 3, 3), 1, 1, 1, groups, dg)

    assert D.fused_ok(geom(64, 64), torch.bfloat16)
    assert D.fused_ok(geom(64, 16, dg=1), torch.bfloat16)
    assert not D.fused_ok(geom(64, 64), torch.float32)      # exact-f32 mode keeps im2col + GEMM
    assert not D.fused_ok(geom(32, 64, dg=4), torch.bfloat16)  # 64 input channels only
    assert not D.fused_ok(geom(64, 128), torch.bfloat16)    # <= 64 outputs
    assert not D.fused_ok(geom(64, 64, groups=2), torch.bfloat16)
    g = geom(64, 128)
    dummy = ctypes.c_void_p(16)
    rc = lib.sr_dcn_fwd_fused(g.desc(torch.bfloat16), dummy, 0, dummy, dummy, dummy, 576, 128, 128, None, dummy,
                              None, None)
    assert rc == -1 and b'unsupported shape' in lib.sr_last_error()
    g = geom(64, 64)
    rc = lib.sr_dcn_fwd_fused(g.desc(torch.bfloat16), dummy, 0, dummy, dummy, dummy, 288, 64, 64, None, dummy,
                              None, None)
    assert rc == -1 and b'weight image' in lib.sr_last_error()


def test_colsum_geometry():
    """Host-side kernel choice behind the fused channel sums (no GPU launch)."""
    from basicsr4rs_amd.ops import conv as C
    lib = _lib.load()
    bf = torch.bfloat16
    # RCAN body conv: band kernel, 8 rows per band (2048 rows over 256 bands) x 2 pixel waves, summed per
    # band (round 6; per row: 64 x 2); variant 37 keeps the per-row sums, and so do one-row bands (B 3: 192
    # rows) and bands that do not divide the image height (B 12: 3 rows per band)
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 32, 64, 64, 64, 64, 64, 64, 64)) == 64 // 8 * 2
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 3, 64, 64, 64, 64, 64, 64, 64)) == 64 * 2
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 12, 64, 64, 64, 64, 64, 64, 64)) == 64 * 2
    try:
        _lib.check(lib.sr_conv3x3_set_variant(37))
        assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 32, 64, 64, 64, 64, 64, 64, 64)) == 64 * 2
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))
    # EDSR-L body conv: 256x256 phase-interleaved kernel, 8 waves per 128-row chunk
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 32, 64, 64, 256, 256, 256, 256, 256)) == 4096 // 128 * 8
    # Cout 16: 256-row chunks of 4 waves
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 2, 16, 16, 64, 64, 16, 16, 16)) == 1 * 4
    # pixel-shuffled store and H*W not a multiple of the chunk: unavailable
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 2, 16, 16, 64, 64, 256, 256, 64, out_ps=2)) == 0
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 2, 10, 10, 64, 64, 64, 64, 64)) == 0
    assert lib.sr_channel_partials_count(4096) == 16 and lib.sr_channel_partials_count(100) == 1


def test_cpu_tensors_refused():
    with pytest.raises(NotImplementedError):
        _lib.ptr(torch.zeros(4))


def test_struct_layouts_match_header():
    # field order / kind / size of the ctypes mirrors vs the C structs (4-byte scalars, 8-byte pointers)
    src = re.sub(r'/\*.*?\*/', '', open(os.path.join(ROOT, 'include', 'sr_hip.h')).read(), flags=re.S)
    for cls, tag in ((_lib.ConvDesc, 'sr_conv3x3_desc'), (_lib.WgradDesc, 'sr_conv3x3_wgrad_desc'),
                     (_lib.DcnDesc, 'sr_dcn_desc')):
        body = re.search(r'typedef struct ' + tag + r' \{(.*?)\}', src, re.S).group(1)
        fields, size, align = [], 0, 4
        for decl in body.split(';'):
            decl = decl.strip()
            if not decl:
                continue
            ptr = '*' in decl
            names = decl.replace('*', ' ').split()[-1] if ptr else decl.split(None, 1)[1]
            for n in names.split(','):
                fields.append((n.strip(), ptr))
                w = 8 if ptr else 4
                size = (size + w - 1) // w * w + w
                align = max(align, w)
        size = (size + align - 1) // align * align
        assert [f[0] for f in cls._fields_] == [n for n, _ in fields]
        assert [f[1] is ctypes.c_void_p for f in cls._fields_] == [p for _, p in fields]
        assert ctypes.sizeof(cls) == size


def test_round3_kernel_selection():
    """Host-side choice of the round-3 kernels (no GPU launch): the 1x1 weight gradient and the streamed
    linear on the SwinIR-M shapes, the row-streaming wgrad over output tiles for 184-channel convs, the
    variant switches that turn each off, and the band kernel's dot-partials query."""
    from basicsr4rs_amd.ops import conv as C
    lib = _lib.load()
    bf = torch.bfloat16

    def wname(cin, cout, ks, N=32, H=64, W=64):
        d = _lib.WgradDesc()
        d.dtype, d.N, d.H, d.W = _lib.dtype_code(bf), N, H, W
        d.Cin, d.Cin_real, d.ldx, d.Cout, d.Cout_real, d.ldy, d.ksize = cin, cin, cin, cout, cout, cout, ks
        return lib.sr_conv3x3_wgrad_kernel_name(d)

    def fname(cin, cout, ks=1):
        return lib.sr_conv3x3_fwd_kernel_name(C._desc(bf, 32, 64, 64, cin, cin, cout, cout, cout, ksize=ks))

    try:
        for cin, cout in ((184, 576), (192, 184), (184, 360), (360, 184)):  # qkv / proj / fc1 / fc2
            assert wname(cin, cout, 1) == b'linear_wgrad_kernel'
        assert wname(184, 184, 3) == b'conv3x3_wgrad_ring_kernel'   # SwinIR RSTB conv
        assert wname(8, 256, 3) == b'conv3x3_wgrad_ring_kernel'     # EDSR conv_first
        assert wname(256, 256, 3) == b'conv3x3_wgrad_row3_kernel'   # EDSR-L body: kernel-row wgrad
        assert wname(128, 512, 3, W=128) == b'conv3x3_wgrad_row3_kernel'
        assert wname(256, 264, 3) != b'conv3x3_wgrad_row3_kernel'   # Cout not a multiple of 256
        for cin, cout in ((576, 184), (360, 184), (184, 360), (184, 184), (192, 184)):
            assert fname(cin, cout) == b'linear_wk_kernel'
        assert fname(184, 576) == b'linear_wk_kernel'                 # qkv unfused (SR_LN_UNFUSED): 3 tiles
        assert fname(184, 640) == b'conv3x3_lin_kernel'               # Cout > 576: lin
        assert fname(384, 40) == b'conv3x3_lin_kernel'                # Cout <= 96: lin
        _lib.check(lib.sr_conv3x3_set_variant(63))
        assert wname(184, 576, 1) == b'conv3x3_wgrad_pp_kernel'
        _lib.check(lib.sr_conv3x3_set_variant(78))
        assert wname(256, 256, 3) == b'conv3x3_wgrad_pp_kernel'     # variant 78: the pp kernel
        _lib.check(lib.sr_conv3x3_set_variant(64))
        assert fname(576, 184) == b'conv3x3_lin_kernel'
        _lib.check(lib.sr_conv3x3_set_variant(62))
        assert lib.sr_conv3x3_get_variant() == 62
        assert wname(256, 256, 3) == b'conv3x3_wgrad_ring_kernel'
        _lib.check(lib.sr_conv3x3_set_variant(0))
        # dot partials: the band kernel's residual + colsum + dot epilogue on the RCAB conv shape only
        assert C.dot_partials_ok(bf, 32, 64, 64, 64, 64)
        assert not C.dot_partials_ok(bf, 32, 64, 64, 64, 32)
        assert not C.dot_partials_ok(torch.float32, 32, 64, 64, 64, 64)
        _lib.check(lib.sr_conv3x3_set_variant(34))
        assert not C.dot_partials_ok(bf, 32, 64, 64, 64, 64)
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))


def test_async_hold_released_at_outermost_exit():
    """The side-stream dy references are dropped when the outermost async_wgrad context exits."""
    from basicsr4rs_amd.ops import conv as C
    dy = torch.zeros(2, 3)
    with C.async_wgrad(True):
        with C.async_wgrad(True):
            C._ASYNC['hold'].append(dy)
        assert C._ASYNC['hold'] == [dy]  # inner exit: still inside the outer backward
    assert C._ASYNC['hold'] == []


def test_strip_band_selection():
    """Host-side choice of the column-strip band kernel (no GPU launch): the RRDBNet HR tail's 64-channel
    convs at W 256 / 512 (with the nearest x2 upsample folded in for conv_up1 / conv_up2), conv_last's
    8-channel dgrad, W 128 with the upsample; widths that are not whole 128-px strips and variant 76 stay
    on the generic tile kernel."""
    from basicsr4rs_amd.ops import conv as C
    lib = _lib.load()
    bf = torch.bfloat16

    def name(N, H, W, cin, cout=64, **kw):
        return lib.sr_conv3x3_fwd_kernel_name(C._desc(bf, N, H, W, cin, cin, cout, cout, cout, **kw))

    band = b'conv3x3_fwd_band_kernel'
    try:
        assert name(16, 512, 512, 64) == band                 # conv_hr and the conv_hr / conv_up2 dgrads
        assert name(16, 512, 512, 64, in_up=2) == band        # conv_up2
        assert name(16, 256, 256, 64, in_up=2) == band        # conv_up1
        assert name(16, 512, 512, 8) == band                  # conv_last dgrad (8 padded channels)
        assert name(32, 256, 256, 8, cout=256) == band        # EDSR conv_last dgrad: one CO 256 launch
        assert lib.sr_conv3x3_fwd_launches(C._desc(bf, 32, 256, 256, 8, 8, 256, 256, 256)) == 1
        assert lib.sr_conv3x3_fwd_launches(C._desc(bf, 32, 256, 256, 8, 8, 192, 192, 192)) == 3  # 64-ch slices
        assert name(32, 256, 256, 64, cout=256) != band       # wide input: stays on the 256-wide kernels
        assert name(2, 256, 256, 256, cout=256) == b'conv3x3_fwd_pph_kernel'  # EDSR body at LR 256: pph strips
        assert name(2, 256, 256, 256, cout=1024, out_ps=2) == b'conv3x3_fwd_pph_kernel'
        assert name(2, 64, 128, 64, in_up=2) == band          # one strip with the upsample
        assert name(2, 96, 96, 64) != band                    # not whole strips
        assert name(2, 64, 256, 64, cout=32) != band          # 64 output channels only
        assert name(2, 64, 256, 40) != band                   # Cin 8..32 or 64
        _lib.check(lib.sr_conv3x3_set_variant(76))
        assert name(16, 512, 512, 64) != band
        _lib.check(lib.sr_conv3x3_set_variant(77))
        assert name(2, 256, 256, 256, cout=256) == b'conv3x3_fwd_pp_kernel'
    finally:
        _lib.check(lib.sr_conv3x3_set_variant(0))


def test_dot_parts_handoff():
    """The RCAB dot-partials hand-off takes the partials only for the same u and an unmodified dy, once."""
    from basicsr4rs_amd.ops import blocks as B
    u, dy, parts = torch.zeros(2, 3), torch.zeros(2, 3), torch.ones(1)
    B._dot_parts_put(dy, parts, u)
    assert B._dot_parts_take(dy, torch.zeros(2, 3)) is None  # another u
    B._dot_parts_put(dy, parts, u)
    dy.add_(1.0)  # an in-place accumulation after the hand-off
    assert B._dot_parts_take(dy, u) is None
    B._dot_parts_put(dy, parts, u)
    assert B._dot_parts_take(dy, u) is parts
    assert B._dot_parts_take(dy, u) is None  # consumed
