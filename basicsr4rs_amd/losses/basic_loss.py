"""Pixel losses (mirror of basicsr/losses/basic_loss.py:12-114, loss_util.py:6-96).

L1Loss with reduction 'mean'/'sum' and no weight map — the configuration of every SR
train YAML on the hot path (e.g. options/train/EDSR/train_EDSR_Lx4.yml ``pixel_opt``) — is
one fused HIP reduction that also writes the gradient (sr_l1_loss).  Weighted or
reduction='none' variants use plain torch ops on the device tensors.
"""
import torch
from torch import nn as nn

from .. import _lib
from ..utils.registry import LOSS_REGISTRY

_reduction_modes = ['none', 'mean', 'sum']


class _L1Fused(torch.autograd.Function):

    @staticmethod
    def forward(ctx, pred, target, loss_weight, mean):
        pred = pred.float().contiguous()
        target = target.float().contiguous()
        lib = _lib.load()
        n = pred.numel()
        ws_bytes = lib.sr_l1_loss_workspace(n)
        ws = torch.empty(ws_bytes // 4 + 1, device=pred.device, dtype=torch.float32)
        loss = torch.empty((), device=pred.device, dtype=torch.float32)
        grad = torch.empty_like(pred) if ctx.needs_input_grad[0] else None
        _lib.check(
            lib.sr_l1_loss(_lib.ptr(pred), _lib.ptr(target), n, float(loss_weight), int(mean), _lib.ptr(loss),
                           _lib.ptr(grad), _lib.ptr(ws), ws_bytes, _lib.stream()))
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad, ) = ctx.saved_tensors
        return grad * g, None, None, None


@LOSS_REGISTRY.register()
class L1Loss(nn.Module):
    """L1 (mean absolute error, MAE) loss (basic_loss.py:27-52)."""

    def __init__(self, loss_weight=1.0, reduction='mean'):
        super().__init__()
        if reduction not in _reduction_modes:
            raise ValueError(f'Unsupported reduction mode: {reduction}. Supported ones are: {_reduction_modes}')
        self.loss_weight = loss_weight
        self.reduction = reduction

    def forward(self, pred, target, weight=None, **kwargs):
        if weight is None and self.reduction in ('mean', 'sum') and pred.is_cuda:
            return _L1Fused.apply(pred, target, self.loss_weight, self.reduction == 'mean')
        if not pred.is_cuda:
            raise NotImplementedError('basicsr4rs_amd losses run on the MI355X device')
        loss = (pred - target).abs()
        if weight is not None:
            loss = loss * weight
        if self.reduction == 'mean':
            # weight_reduce_loss (loss_util.py:32-56): mean over weighted elements
            loss = loss.mean() if weight is None else loss.sum() / (weight.sum() if weight.size(1) > 1 else weight.sum() * loss.size(1))
        elif self.reduction == 'sum':
            loss = loss.sum()
        return self.loss_weight * loss
