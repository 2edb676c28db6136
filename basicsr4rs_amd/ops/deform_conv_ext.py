"""``deform_conv_ext`` drop-in: the five pybind functions of basicsr/ops/dcn/src/deform_conv_ext.cpp
(:151-163) over the C ABI of csrc/dcn_ext.hip.

Same names, same positional arguments in the same order, same buffer semantics (caller-owned,
zero-initialised grads accumulated into; output overwritten; ``columns`` / ``ones`` accepted and
not needed), same return values (1 for the ``int`` functions, None for the ``void`` ones).  So
the reference's own ``basicsr/ops/dcn/deform_conv.py`` runs unchanged with
``from basicsr4rs_amd.ops import deform_conv_ext``.  Tensors: fp32, CUDA (HIP),
contiguous NCHW, like the reference's float path; CPU tensors raise NotImplementedError and a
failed check raises RuntimeError (TORCH_CHECK / AT_ERROR in the reference).
"""
import torch

from .. import _lib

__all__ = ['deform_conv_forward', 'deform_conv_backward_input', 'deform_conv_backward_parameters',
           'modulated_deform_conv_forward', 'modulated_deform_conv_backward']


def _check(*tensors):
    for t in tensors:
        if not t.is_cuda:
            raise NotImplementedError('deform conv is not implemented on CPU')
        if t.dtype != torch.float32:
            raise RuntimeError(f'deform_conv_ext (HIP): float32 tensors expected, got {t.dtype}')
        if not t.is_contiguous():
            raise RuntimeError('deform_conv_ext (HIP): contiguous tensors expected')


def _sizes(input, weight):
    if input.dim() != 4:
        raise RuntimeError(f'deform_conv_ext (HIP): 4-D NCHW input expected, got {input.dim()}-D')
    n, c, h, w = input.shape
    return [int(n), int(c), int(h), int(w), int(weight.size(0))]


def _workspace(sizes, geo, step):
    lib = _lib.load()
    nbytes = lib.sr_deform_conv_workspace(*sizes, *geo, step)
    if nbytes == 0:
        raise RuntimeError(f'deform_conv_ext: {lib.sr_last_error().decode()}')
    return torch.empty(nbytes // 4 + 1, device=torch.cuda.current_device(), dtype=torch.float32), nbytes


def deform_conv_forward(input, weight, offset, output, columns, ones, kW, kH, dW, dH, padW, padH, dilationW,
                        dilationH, group, deformable_group, im2col_step):
    _check(input, weight, offset, output)
    sz = _sizes(input, weight)
    geo = [kW, kH, dW, dH, padW, padH, dilationW, dilationH, group, deformable_group]
    ws, nb = _workspace(sz, geo, im2col_step)
    lib = _lib.load()
    _lib.check(lib.sr_deform_conv_forward(_lib.ptr(input), _lib.ptr(weight), _lib.ptr(offset), _lib.ptr(output), None,
                                          None, *sz, *geo, im2col_step, _lib.ptr(ws), nb, _lib.stream()))
    return 1


def deform_conv_backward_input(input, offset, gradOutput, gradInput, gradOffset, weight, columns, kW, kH, dW, dH, padW,
                               padH, dilationW, dilationH, group, deformable_group, im2col_step):
    gradOutput = gradOutput.contiguous()
    _check(input, offset, gradOutput, gradInput, gradOffset, weight)
    sz = _sizes(input, weight)
    geo = [kW, kH, dW, dH, padW, padH, dilationW, dilationH, group, deformable_group]
    ws, nb = _workspace(sz, geo, im2col_step)
    lib = _lib.load()
    _lib.check(
        lib.sr_deform_conv_backward_input(_lib.ptr(input), _lib.ptr(offset), _lib.ptr(gradOutput), _lib.ptr(gradInput),
                                          _lib.ptr(gradOffset), _lib.ptr(weight), None, *sz, *geo, im2col_step,
                                          _lib.ptr(ws), nb, _lib.stream()))
    return 1


def deform_conv_backward_parameters(input, offset, gradOutput, gradWeight, columns, ones, kW, kH, dW, dH, padW, padH,
                                    dilationW, dilationH, group, deformable_group, scale, im2col_step):
    gradOutput = gradOutput.contiguous()
    _check(input, offset, gradOutput, gradWeight)
    sz = _sizes(input, gradWeight)
    geo = [kW, kH, dW, dH, padW, padH, dilationW, dilationH, group, deformable_group]
    ws, nb = _workspace(sz, geo, im2col_step)
    lib = _lib.load()
    _lib.check(
        lib.sr_deform_conv_backward_parameters(_lib.ptr(input), _lib.ptr(offset), _lib.ptr(gradOutput),
                                               _lib.ptr(gradWeight), None, None, *sz, *geo, float(scale), im2col_step,
                                               _lib.ptr(ws), nb, _lib.stream()))
    return 1


def _mgeo(kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, group, deformable_group):
    # the workspace query takes the v1 order (kW, kH, dW, dH, padW, padH, dilW, dilH, ...)
    return [kernel_w, kernel_h, stride_w, stride_h, pad_w, pad_h, dilation_w, dilation_h, group, deformable_group]


def modulated_deform_conv_forward(input, weight, bias, ones, offset, mask, output, columns, kernel_h, kernel_w,
                                  stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, group, deformable_group,
                                  with_bias):
    _check(input, weight, offset, mask, output)
    if with_bias:
        _check(bias)
    sz = _sizes(input, weight)
    ws, nb = _workspace(sz, _mgeo(kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, group,
                                  deformable_group), sz[0])
    lib = _lib.load()
    _lib.check(
        lib.sr_modulated_deform_conv_forward(_lib.ptr(input), _lib.ptr(weight), _lib.ptr(bias) if with_bias else None,
                                             None, _lib.ptr(offset), _lib.ptr(mask), _lib.ptr(output), None, *sz,
                                             kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h,
                                             dilation_w, group, deformable_group, int(bool(with_bias)), _lib.ptr(ws),
                                             nb, _lib.stream()))


def modulated_deform_conv_backward(input, weight, bias, ones, offset, mask, columns, grad_input, grad_weight,
                                   grad_bias, grad_offset, grad_mask, grad_output, kernel_h, kernel_w, stride_h,
                                   stride_w, pad_h, pad_w, dilation_h, dilation_w, group, deformable_group, with_bias):
    grad_output = grad_output.contiguous()
    _check(input, weight, offset, mask, grad_input, grad_weight, grad_offset, grad_mask, grad_output)
    if with_bias:
        _check(grad_bias)
    sz = _sizes(input, weight)
    ws, nb = _workspace(sz, _mgeo(kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, group,
                                  deformable_group), sz[0])
    lib = _lib.load()
    _lib.check(
        lib.sr_modulated_deform_conv_backward(_lib.ptr(input), _lib.ptr(weight), None, None, _lib.ptr(offset),
                                              _lib.ptr(mask), None, _lib.ptr(grad_input), _lib.ptr(grad_weight),
                                              _lib.ptr(grad_bias) if with_bias else None, _lib.ptr(grad_offset),
                                              _lib.ptr(grad_mask), _lib.ptr(grad_output), *sz, kernel_h, kernel_w,
                                              stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w, group,
                                              deformable_group, int(bool(with_bias)), _lib.ptr(ws), nb, _lib.stream()))
