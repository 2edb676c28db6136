"""ORACLE — numpy restatement of the validation arithmetic (test infrastructure only; the product
path never imports it).

* ``minusone_one_to_ubyte``: basicsr/utils/img_util.py:99-128 — clamp to [-1, 1], (x + 1) / 2,
  torchvision ``make_grid(t, nrow=B, normalize=True, value_range=(0, 1))`` (1-channel maps
  repeated to 3, one image returned as is, else a 2-px zero-padded row of tiles), CHW -> HWC,
  skimage ``img_as_ubyte`` (float32 x * 255, round half to even, clip).
* ``psnr``: basicsr/metrics/psnr_ssim.py:11-48 (HWC, crop, float64 MSE, 10 log10(255^2 / MSE)).

Written from the published behaviour of those calls with explicit loops / numpy, independent of
the product's torch-based helpers.
"""
import numpy as np


def minusone_one_to_ubyte(x):
    """x: float array [B, C, H, W] -> uint8 [H', W', C'] (see module docstring)."""
    x = np.asarray(x, dtype=np.float32)
    x = (np.clip(x, -1.0, 1.0) + np.float32(1.0)) / np.float32(2.0)
    if x.shape[1] == 1:
        x = np.concatenate([x, x, x], axis=1)
    x = np.clip(x, 0.0, 1.0)
    B, C, H, W = x.shape
    if B == 1:
        grid = x[0]
    else:
        pad = 2
        grid = np.zeros((C, H + 2 * pad, B * (W + pad) + pad), dtype=np.float32)
        for b in range(B):
            x0 = b * (W + pad) + pad
            grid[:, pad:pad + H, x0:x0 + W] = x[b]
    img = grid.transpose(1, 2, 0)
    out = np.rint(img * np.float32(255.0)).astype(np.float32)
    return np.clip(out, 0, 255).astype(np.uint8)


def psnr(img, img2, crop_border):
    img = np.asarray(img, dtype=np.float64)
    img2 = np.asarray(img2, dtype=np.float64)
    if crop_border:
        img = img[crop_border:-crop_border, crop_border:-crop_border, ...]
        img2 = img2[crop_border:-crop_border, crop_border:-crop_border, ...]
    mse = float(np.mean((img - img2)**2))
    return float('inf') if mse == 0 else 10.0 * np.log10(255.0 * 255.0 / mse)
