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


def test_colsum_geometry():
    """Host-side kernel choice behind the fused channel sums (no GPU launch)."""
    from basicsr4rs_amd.ops import conv as C
    lib = _lib.load()
    bf = torch.bfloat16
    # RCAN body conv: narrow halo kernel, 128-row epilogue chunks x 4 waves
    assert lib.sr_conv3x3_fwd_colsum_parts(C._desc(bf, 32, 64, 64, 64, 64, 64, 64, 64)) == 4096 // 128 * 4
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
