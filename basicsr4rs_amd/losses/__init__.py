"""Loss registry surface (mirror of basicsr/losses/__init__.py:19-31)."""
from copy import deepcopy

from ..utils.registry import LOSS_REGISTRY
from .basic_loss import L1Loss

__all__ = ['build_loss', 'L1Loss']


def build_loss(opt):
    opt = deepcopy(opt)
    loss_type = opt.pop('type')
    return LOSS_REGISTRY.get(loss_type)(**opt)
