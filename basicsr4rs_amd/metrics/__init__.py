"""Metric registry surface (mirror of basicsr/metrics/__init__.py:11-21)."""
from copy import deepcopy

from ..utils.registry import METRIC_REGISTRY
from .psnr_ssim import calculate_psnr, calculate_psnr_pt, calculate_ssim, calculate_ssim_pt

__all__ = ['calculate_psnr', 'calculate_psnr_pt', 'calculate_ssim', 'calculate_ssim_pt', 'calculate_metric']


def calculate_metric(data, opt):
    opt = deepcopy(opt)
    metric_type = opt.pop('type')
    return METRIC_REGISTRY.get(metric_type)(**data, **opt)
