"""ctypes binding of the C ABI in include/sr_hip.h (libsr_hip.so, gfx950).

The product path calls the HIP kernels only through this module.  There is no CPU or
PyTorch fallback: if the shared library is missing or a tensor is not on the GPU the call
raises, like the reference's extension ops (basicsr/ops/dcn/deform_conv.py:61-62 raises
NotImplementedError for CPU tensors; TORCH_CHECK failures surface as RuntimeError).
"""
import ctypes
import os

import torch

from ._switches import switch

LIB_PATH = switch('SR_HIP_LIB') or os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib',
                                                         'libsr_hip.so')

SR_F32, SR_BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t


class ConvDesc(ctypes.Structure):
    _fields_ = [('dtype', _i), ('N', _i), ('H', _i), ('W', _i), ('Cin', _i), ('ldx', _i), ('xcoff', _i),
                ('in_ps', _i), ('Cout', _i), ('Cout_real', _i), ('ldw', _i), ('ldy', _i), ('ycoff', _i),
                ('out_ps', _i), ('out_nchw', _i), ('act', _i), ('slope', _f), ('alpha', _f), ('ldg', _i),
                ('gcoff', _i), ('gate_slope', _f), ('ldr', _i), ('rcoff', _i), ('beta', _f), ('ldr2', _i),
                ('r2coff', _i), ('beta2', _f), ('rcols', _i), ('in_up', _i), ('ksize', _i), ('gate_mode', _i),
                ('gcol0', _i), ('gcol1', _i), ('row_scale', _vp), ('dot', _vp), ('ldd', _i), ('dcoff', _i)]


class WgradDesc(ctypes.Structure):
    _fields_ = [('dtype', _i), ('N', _i), ('H', _i), ('W', _i), ('Cin', _i), ('Cin_real', _i), ('ldx', _i),
                ('xcoff', _i), ('Cout', _i), ('Cout_real', _i), ('ldy', _i), ('ycoff', _i), ('out_ps', _i),
                ('scale', _f), ('in_up', _i), ('ksize', _i), ('accumulate', _i)]


class PrepItem(ctypes.Structure):
    _fields_ = [('w', _vp), ('bias', _vp), ('Cout_real', _i), ('Cin_real', _i), ('Cout', _i), ('Cin', _i),
                ('out_ps', _i), ('ksize', _i), ('row_map', _vp), ('col_map', _vp), ('wf', _vp), ('wd', _vp),
                ('bias_g', _vp)]


class DcnDesc(ctypes.Structure):
    _fields_ = [('dtype', _i), ('N', _i), ('C', _i), ('H', _i), ('W', _i), ('Cp', _i), ('Ho', _i), ('Wo', _i),
                ('kh', _i), ('kw', _i), ('stride_h', _i), ('stride_w', _i), ('pad_h', _i), ('pad_w', _i),
                ('dil_h', _i), ('dil_w', _i), ('groups', _i), ('deformable_groups', _i), ('cgp', _i)]


# name -> (restype, argtypes); must match include/sr_hip.h (checked by tests/test_abi.py)
SIGNATURES = {
    'sr_version': (ctypes.c_char_p, []),
    'sr_last_error': (ctypes.c_char_p, []),
    'sr_set_knob': (_i, [ctypes.c_char_p, _i, ctypes.POINTER(_i)]),
    'sr_get_knob': (_i, [ctypes.c_char_p]),
    'sr_conv3x3_fwd': (_i, [ctypes.POINTER(ConvDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'sr_linear_ln_fwd': (_i, [ctypes.POINTER(ConvDesc), _vp, _vp, _vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'sr_conv3x3_fwd_colsum_parts': (_i, [ctypes.POINTER(ConvDesc)]),
    'sr_conv3x3_fwd_dot_ok': (_i, [ctypes.POINTER(ConvDesc)]),
    'sr_conv3x3_get_variant': (_i, []),
    'sr_conv3x3_set_variant': (_i, [_i]),
    'sr_conv3x3_set_stamps': (_i, [_vp]),
    'sr_conv3x3_fwd_kernel_name': (ctypes.c_char_p, [ctypes.POINTER(ConvDesc)]),
    'sr_conv3x3_fwd_launches': (_i, [ctypes.POINTER(ConvDesc)]),
    'sr_conv3x3_wgrad_kernel_name': (ctypes.c_char_p, [ctypes.POINTER(WgradDesc)]),
    'sr_conv3x3_wgrad_workspace': (_sz, [ctypes.POINTER(WgradDesc)]),
    'sr_conv3x3_wgrad': (_i, [ctypes.POINTER(WgradDesc), _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp]),
    'sr_conv3x3_wgrad_reduce': (_i, [ctypes.POINTER(WgradDesc), _vp, _sz, _vp, _vp, _vp, _vp, _vp]),
    'sr_conv_prep_blocks': (_i, [ctypes.POINTER(PrepItem)]),
    'sr_conv_prep_batch': (_i, [_i, _vp, _vp, _i, _i, _vp]),
    'sr_conv3x3_prep': (_i, [_i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    'sr_conv_prep_mapped': (_i, [_i, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    'sr_nchw_to_nhwc': (_i, [_i, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    'sr_nhwc_to_nchw': (_i, [_i, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    'sr_pixel_shuffle_nchw': (_i, [_i, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    'sr_l1_loss': (_i, [_vp, _vp, _i64, _f, _i, _vp, _vp, _vp, _sz, _vp]),
    'sr_l1_loss_workspace': (_sz, [_i64]),
    'sr_act_backward': (_i, [_i, _vp, _vp, _i64, _i, _f, _f, _vp, _vp]),
    'sr_row_scale': (_i, [_i, _vp, _i64, _i, _i, _vp, _vp, _vp]),
    'sr_adam_ema': (_i, [_vp, _vp, _vp, _vp, _vp, _i64, _f, _f, _f, _f, _f, _f, _f, _f, _vp]),
    'sr_adam_ema_dev': (_i, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _f, _f, _f, _f, _vp]),
    'sr_bilinear_up_add': (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp]),
    'sr_channel_reduce_workspace': (_sz, [_i, _i, _i]),
    'sr_channel_reduce': (_i, [_i, _vp, _i, _i, _vp, _i, _i, _i, _i, _i, _f, _vp, _vp, _sz, _vp]),
    'sr_channel_partials_count': (_i, [_i]),
    'sr_channel_partials': (_i, [_i, _vp, _i, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    'sr_ca_mlp_fwd': (_i, [_vp, _i, _f, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    'sr_ca_mlp_bwd': (_i, [_vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp]),
    'sr_nc_affine': (_i, [_i, _vp, _vp, _vp, _vp, _i, _i, _i, _f, _f, _f, _vp, _vp]),
    'sr_ca_fwd_apply': (_i, [_i, _vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp,
                             _vp]),
    'sr_ca_bwd_apply': (_i, [_i, _vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    'sr_ca_param_grad': (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp]),
    'sr_act_backward_nhwc': (_i, [_i, _i64, _i, _vp, _i, _i, _vp, _i, _i, _vp, _i, _i, _i, _f, _f, _vp]),
    'sr_nearest_up_backward': (_i, [_i, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _vp]),
    'sr_nearest_up_backward_gate': (_i, [_i, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _f, _vp, _i, _i, _vp]),
    'sr_copy_channels': (_i, [_i, _vp, _i, _i, _vp, _i, _i, _i64, _i, _vp]),
    'sr_layernorm_fwd': (_i, [_i, _vp, _i, _vp, _vp, _i64, _i, _i, _f, _vp, _i, _vp, _vp, _vp]),
    'sr_layernorm_bwd_workspace': (_sz, [_i64, _i]),
    'sr_layernorm_bwd': (_i, [_i, _vp, _i, _vp, _i, _vp, _vp, _vp, _i64, _i, _i, _vp, _i, _vp, _i, _vp, _vp, _vp, _sz,
                             _i, _vp]),
    'sr_window_attn_fwd': (_i, [_i, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _f, _vp, _vp, _i, _vp, _vp]),
    'sr_layernorm_bwd_scaled': (_i, [_i, _vp, _i, _vp, _i, _vp, _vp, _vp, _i64, _i, _i, _vp, _i, _vp, _i, _vp, _vp, _vp, _sz,
                                     _i, _vp, _i, _vp, _vp]),
    'sr_layernorm_bwd_parts': (_i, [_i, _i64, _i, _i, _i, _i, _i]),
    'sr_layernorm_bwd_reduce': (_i, [_vp, _i, _i, _vp, _vp, _i, _vp]),
    'sr_window_attn_bwd_parts': (_i, [_i, _i, _i, _i, _i, _i, _i, _i, _i, _i]),
    'sr_window_attn_dbias_reduce': (_i, [_vp, _i, _i, _i, _vp, _i, _vp]),
    'sr_swin_attn_fused_ok': (_i, [_i, _i, _i, _i, _i, _i, _i, _i, _i, _i]),
    'sr_swin_attn_fused_fwd': (_i, [_vp, _vp, _vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _f, _vp,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'sr_swin_mlp_fused_ok': (_i, [_i, _i, _i, _i]),
    'sr_swin_mlp_fused_fwd': (_i, [_vp, _vp, _vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp,
                                  _vp, _vp, _vp]),
    'sr_window_attn_bwd_workspace': (_sz, [_i, _i, _i, _i, _i]),
    'sr_window_attn_bwd': (_i, [_i, _vp, _i, _vp, _vp, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp,
                               _sz, _i, _vp]),
    'sr_add_pos_embed': (_i, [_i, _vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    'sr_pos_embed_grad': (_i, [_i, _vp, _i, _i, _i, _i, _vp, _i, _vp]),
    'sr_dcn_im2col': (_i, [ctypes.POINTER(DcnDesc), _vp, _vp, _vp, _vp, _vp]),
    'sr_dcn_fwd_fused_ok': (_i, [ctypes.POINTER(DcnDesc), _i]),
    'sr_dcn_fwd_fused': (_i, [ctypes.POINTER(DcnDesc), _vp, _i, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    'sr_dcn_col2im_workspace': (_sz, [ctypes.POINTER(DcnDesc)]),
    'sr_dcn_col2im': (_i, [ctypes.POINTER(DcnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    'sr_dcn_bwd_fused_ok': (_i, [ctypes.POINTER(DcnDesc), _i]),
    'sr_dcn_bwd_fused': (_i, [ctypes.POINTER(DcnDesc), _vp, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp,
                              _sz, _vp]),
    'sr_deform_conv_workspace': (_sz, [_i] * 16),
    'sr_deform_conv_forward': (_i, [_vp] * 6 + [_i] * 16 + [_vp, _sz, _vp]),
    'sr_deform_conv_backward_input': (_i, [_vp] * 7 + [_i] * 16 + [_vp, _sz, _vp]),
    'sr_deform_conv_backward_parameters': (_i, [_vp] * 6 + [_i] * 15 + [_f, _i, _vp, _sz, _vp]),
    'sr_modulated_deform_conv_forward': (_i, [_vp] * 8 + [_i] * 16 + [_vp, _sz, _vp]),
    'sr_modulated_deform_conv_backward': (_i, [_vp] * 13 + [_i] * 16 + [_vp, _sz, _vp]),
    'sr_fused_bias_act': (_i, [_i, _vp, _vp, _vp, _vp, _i64, _i, _i, _i, _i, _f, _f, _vp]),
    'sr_fused_lrelu_bwd_workspace': (_sz, [_i, _i, _i64]),
    'sr_fused_lrelu_bwd': (_i, [_i, _vp, _vp, _vp, _vp, _i, _i, _i64, _f, _f, _vp, _sz, _vp]),
    'sr_upfirdn2d_out_size': (_i, [_i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    'sr_upfirdn2d': (_i, [_i, _vp, _i, _i, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
}

_LIB = None


def load():
    """Load libsr_hip.so once; raise loudly if it was not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f'libsr_hip.so not found at {LIB_PATH}; build it with '
                              '`python -c "import __graft_entry__ as g; g.build()"` or `make -C basicsr4rs_amd/csrc`')
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
        # SR_CONV_VARIANT=<n>: a kernel-selection variant for the whole process (A/B runs,
        # tools/ab_val.sh); 0 / unset = automatic
        v = int(switch('SR_CONV_VARIANT') or 0)
        if v:
            check(lib.sr_conv3x3_set_variant(v))
    return _LIB


class knob:
    """Context: set a library tuning knob (sr_set_knob; the environment variable of the same name
    read once per process) for the block, restoring the previous value on exit."""

    def __init__(self, name, value):
        self.name, self.value, self.prev = name.encode(), int(value), None

    def __enter__(self):
        prev = ctypes.c_int(0)
        check(load().sr_set_knob(self.name, self.value, ctypes.byref(prev)))
        self.prev = prev.value
        return self

    def __exit__(self, *exc):
        check(load().sr_set_knob(self.name, self.prev, None))
        return False


def check(rc):
    if rc != 0:
        raise RuntimeError(f'libsr_hip: {load().sr_last_error().decode()} (status {rc})')


def stream():
    return _vp(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Refuses CPU tensors: no CPU path."""
    if t is None:
        return None
    if not t.is_cuda:
        raise NotImplementedError('basicsr4rs_amd HIP ops need tensors on the MI355X (cuda) device')
    return _vp(t.data_ptr())


def dtype_code(dt):
    if dt == torch.bfloat16:
        return SR_BF16
    if dt == torch.float32:
        return SR_F32
    raise TypeError(f'unsupported feature dtype {dt}')
