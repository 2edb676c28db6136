"""PSNR (mirror of basicsr/metrics/psnr_ssim.py:11-48 and the tensor form :91-121)."""
import numpy as np
import torch

from ..utils.registry import METRIC_REGISTRY


def _reorder(img, input_order):
    if input_order not in ['HWC', 'CHW']:
        raise ValueError(f'Wrong input_order {input_order}. Supported input_orders are "HWC" and "CHW"')
    if img.ndim == 2:
        return img[..., None]
    return img.transpose(1, 2, 0) if input_order == 'CHW' else img


def _to_y(img):
    """BGR uint8-range image -> Y of YCbCr (ITU-R BT.601), as basicsr/metrics/metric_util.py."""
    img = img.astype(np.float32) / 255.
    if img.ndim == 3 and img.shape[2] == 3:
        img = np.dot(img, [24.966, 128.553, 65.481]) + 16.0
        img = img[..., None]
    return img * 255. / 255.


@METRIC_REGISTRY.register()
def calculate_psnr(img, img2, crop_border, input_order='HWC', test_y_channel=False, **kwargs):
    """10*log10(255^2 / MSE) in float64 over the cropped images; inf when identical."""
    assert img.shape == img2.shape, f'Image shapes are different: {img.shape}, {img2.shape}.'
    img = _reorder(img, input_order)
    img2 = _reorder(img2, input_order)
    if crop_border != 0:
        img = img[crop_border:-crop_border, crop_border:-crop_border, ...]
        img2 = img2[crop_border:-crop_border, crop_border:-crop_border, ...]
    if test_y_channel:
        img, img2 = _to_y(img), _to_y(img2)
    mse = np.mean((img.astype(np.float64) - img2.astype(np.float64))**2)
    if mse == 0:
        return float('inf')
    return 10. * np.log10(255. * 255. / mse)


@METRIC_REGISTRY.register()
def calculate_psnr_pt(img, img2, crop_border, test_y_channel=False, **kwargs):
    """Tensor PSNR on [0,1] NCHW images, per image (psnr_ssim.py:91-121)."""
    assert img.shape == img2.shape, f'Image shapes are different: {img.shape}, {img2.shape}.'
    if crop_border != 0:
        img = img[:, :, crop_border:-crop_border, crop_border:-crop_border]
        img2 = img2[:, :, crop_border:-crop_border, crop_border:-crop_border]
    if test_y_channel:
        w = torch.tensor([65.481, 128.553, 24.966], device=img.device, dtype=img.dtype).view(1, 3, 1, 1)
        img = ((img * w).sum(1, keepdim=True) + 16.0) / 255.
        img2 = ((img2 * w).sum(1, keepdim=True) + 16.0) / 255.
    img = img.to(torch.float64)
    img2 = img2.to(torch.float64)
    mse = torch.mean((img - img2)**2, dim=[1, 2, 3])
    return 10. * torch.log10(1. / (mse + 1e-8))
