"""PSNR / SSIM (mirror of basicsr/metrics/psnr_ssim.py:11-48, :91-121, :125-170, :210-309).

Validation-side host metrics (numpy / torch), not the train hot path.  The reference's SSIM
filters with OpenCV (cv2.getGaussianKernel(11, 1.5), cv2.filter2D, then the valid 5-pixel
crop, psnr_ssim.py:261-276); cv2 is not in this image, so the same 11x11 Gaussian window is
built from its closed form and applied as a separable valid-mode correlation -- identical in
the cropped region, where the border mode of filter2D never reaches.
"""
import numpy as np
import torch
from torch.nn import functional as F

from ..utils.registry import METRIC_REGISTRY


def _reorder(img, input_order):
    if input_order not in ['HWC', 'CHW']:
        raise ValueError(f'Wrong input_order {input_order}. Supported input_orders are "HWC" and "CHW"')
    if img.ndim == 2:
        return img[..., None]
    return img.transpose(1, 2, 0) if input_order == 'CHW' else img


def _to_y(img):
    """to_y_channel (basicsr/metrics/metric_util.py:32-45): BGR [0,255] image -> Y of YCbCr
    (ITU-R BT.601, bgr2ycbcr(y_only=True), basicsr/utils/color_util.py:38-68), [0,255] float."""
    img = img.astype(np.float32) / 255.
    if img.ndim == 3 and img.shape[2] == 3:
        y = np.dot(img, [24.966, 128.553, 65.481]) + 16.0
        img = (y / 255.).astype(np.float32)[..., None]
    return img * 255.


def _rgb2y_pt(img):
    """rgb2ycbcr_pt(y_only=True) (basicsr/utils/color_util.py:186-208): [0,1] RGB -> [0,1] Y."""
    w = torch.tensor([[65.481], [128.553], [24.966]]).to(img)
    return (torch.matmul(img.permute(0, 2, 3, 1), w).permute(0, 3, 1, 2) + 16.0) / 255.


def gaussian_window(ksize=11, sigma=1.5):
    """cv2.getGaussianKernel(ksize, sigma) (float64, normalised to sum 1) outer itself."""
    x = np.arange(ksize, dtype=np.float64) - (ksize - 1) * 0.5
    k = np.exp(-x * x / (2.0 * sigma * sigma))
    k = (k / k.sum()).reshape(-1, 1)
    return k @ k.T


def _filter_valid(img, k1):
    """Valid-mode correlation of a 2-D float64 image with the separable window k1 x k1^T."""
    n = k1.shape[0]
    h, w = img.shape
    t = np.zeros((h - n + 1, w), dtype=np.float64)
    for i in range(n):
        t += k1[i] * img[i:i + h - n + 1, :]
    out = np.zeros((h - n + 1, w - n + 1), dtype=np.float64)
    for j in range(n):
        out += k1[j] * t[:, j:j + w - n + 1]
    return out


def _ssim(img, img2):
    """SSIM of one channel in [0,255] (psnr_ssim.py:248-276)."""
    c1 = (0.01 * 255)**2
    c2 = (0.03 * 255)**2
    if img.shape[0] < 11 or img.shape[1] < 11:
        return np.nan  # the reference's [5:-5, 5:-5] crop of the filtered map is empty: mean = nan
    x = np.arange(11, dtype=np.float64) - 5.0
    k1 = np.exp(-x * x / (2.0 * 1.5 * 1.5))
    k1 /= k1.sum()
    mu1 = _filter_valid(img, k1)
    mu2 = _filter_valid(img2, k1)
    mu1_sq, mu2_sq, mu1_mu2 = mu1**2, mu2**2, mu1 * mu2
    sigma1_sq = _filter_valid(img**2, k1) - mu1_sq
    sigma2_sq = _filter_valid(img2**2, k1) - mu2_sq
    sigma12 = _filter_valid(img * img2, k1) - mu1_mu2
    ssim_map = ((2 * mu1_mu2 + c1) * (2 * sigma12 + c2)) / ((mu1_sq + mu2_sq + c1) * (sigma1_sq + sigma2_sq + c2))
    return ssim_map.mean()


def _ssim_pth(img, img2):
    """SSIM per image of [n, c, h, w] tensors in [0,255] (psnr_ssim.py:279-309)."""
    c1 = (0.01 * 255)**2
    c2 = (0.03 * 255)**2
    window = torch.from_numpy(gaussian_window()).view(1, 1, 11, 11).expand(img.size(1), 1, 11, 11)
    window = window.to(img.dtype).to(img.device)
    conv = lambda t: F.conv2d(t, window, stride=1, padding=0, groups=img.shape[1])  # noqa: E731
    mu1, mu2 = conv(img), conv(img2)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = conv(img * img) - mu1_sq
    sigma2_sq = conv(img2 * img2) - mu2_sq
    sigma12 = conv(img * img2) - mu1_mu2
    cs_map = (2 * sigma12 + c2) / (sigma1_sq + sigma2_sq + c2)
    ssim_map = ((2 * mu1_mu2 + c1) / (mu1_sq + mu2_sq + c1)) * cs_map
    return ssim_map.mean([1, 2, 3])


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
        img, img2 = _rgb2y_pt(img), _rgb2y_pt(img2)
    img = img.to(torch.float64)
    img2 = img2.to(torch.float64)
    mse = torch.mean((img - img2)**2, dim=[1, 2, 3])
    return 10. * torch.log10(1. / (mse + 1e-8))


@METRIC_REGISTRY.register()
def calculate_ssim(img, img2, crop_border, input_order='HWC', test_y_channel=False, **kwargs):
    """Mean over channels of the single-channel SSIM on [0,255] images (psnr_ssim.py:125-168)."""
    assert img.shape == img2.shape, f'Image shapes are different: {img.shape}, {img2.shape}.'
    img = _reorder(img, input_order)
    img2 = _reorder(img2, input_order)
    if crop_border != 0:
        img = img[crop_border:-crop_border, crop_border:-crop_border, ...]
        img2 = img2[crop_border:-crop_border, crop_border:-crop_border, ...]
    if test_y_channel:
        img, img2 = _to_y(img), _to_y(img2)
    img = img.astype(np.float64)
    img2 = img2.astype(np.float64)
    return np.array([_ssim(img[..., i], img2[..., i]) for i in range(img.shape[2])]).mean()


@METRIC_REGISTRY.register()
def calculate_ssim_pt(img, img2, crop_border, test_y_channel=False, **kwargs):
    """Tensor SSIM on [0,1] NCHW images, per image (psnr_ssim.py:210-245)."""
    assert img.shape == img2.shape, f'Image shapes are different: {img.shape}, {img2.shape}.'
    if crop_border != 0:
        img = img[:, :, crop_border:-crop_border, crop_border:-crop_border]
        img2 = img2[:, :, crop_border:-crop_border, crop_border:-crop_border]
    if test_y_channel:
        img, img2 = _rgb2y_pt(img), _rgb2y_pt(img2)
    img = img.to(torch.float64)
    img2 = img2.to(torch.float64)
    return _ssim_pth(img * 255., img2 * 255.)
