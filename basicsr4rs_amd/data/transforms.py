"""Paired crop / flip / rotation augmentation (basicsr/data/transforms.py:8-228), numpy HWC or
tensor (..., C, H, W) inputs, Python ``random`` as the source of randomness like the reference
(so a seeded worker reproduces the same crops).  Flips are numpy views + copies instead of
cv2.flip (OpenCV is not in this image)."""
import random

import numpy as np
import torch


def mod_crop(img, scale):
    img = img.copy()
    if img.ndim not in (2, 3):
        raise ValueError(f'Wrong img ndim: {img.ndim}.')
    h, w = img.shape[0], img.shape[1]
    return img[:h - h % scale, :w - w % scale, ...]


def paired_random_crop(img_gts, img_lqs, gt_patch_size, scale, gt_path=None):
    """Crop an LQ patch of gt_patch_size // scale at a random position and the GT patch at
    scale x that position; lists are cropped at the same place."""
    if not isinstance(img_gts, list):
        img_gts = [img_gts]
    if not isinstance(img_lqs, list):
        img_lqs = [img_lqs]
    tensor = torch.is_tensor(img_gts[0])
    if tensor:
        h_lq, w_lq = img_lqs[0].size()[-2:]
        h_gt, w_gt = img_gts[0].size()[-2:]
    else:
        h_lq, w_lq = img_lqs[0].shape[0:2]
        h_gt, w_gt = img_gts[0].shape[0:2]
    lq_patch = gt_patch_size // scale
    if h_gt != h_lq * scale or w_gt != w_lq * scale:
        raise ValueError(f'Scale mismatches. GT ({h_gt}, {w_gt}) is not {scale}x multiplication of LQ ({h_lq}, '
                         f'{w_lq}).')
    if h_lq < lq_patch or w_lq < lq_patch:
        raise ValueError(f'LQ ({h_lq}, {w_lq}) is smaller than patch size ({lq_patch}, {lq_patch}). '
                         f'Please remove {gt_path}.')
    top = random.randint(0, h_lq - lq_patch)
    left = random.randint(0, w_lq - lq_patch)
    tg, lg = int(top * scale), int(left * scale)
    if tensor:
        img_lqs = [v[..., top:top + lq_patch, left:left + lq_patch] for v in img_lqs]
        img_gts = [v[..., tg:tg + gt_patch_size, lg:lg + gt_patch_size] for v in img_gts]
    else:
        img_lqs = [v[top:top + lq_patch, left:left + lq_patch, ...] for v in img_lqs]
        img_gts = [v[tg:tg + gt_patch_size, lg:lg + gt_patch_size, ...] for v in img_gts]
    return (img_gts[0] if len(img_gts) == 1 else img_gts), (img_lqs[0] if len(img_lqs) == 1 else img_lqs)


def augment(imgs, hflip=True, rotation=True, flows=None, return_status=False):
    """Horizontal flip and/or rotation by 0/90/180/270 degrees (vertical flip + transpose),
    the same draw for every image (and flow) of the list."""
    hflip = hflip and random.random() < 0.5
    vflip = rotation and random.random() < 0.5
    rot90 = rotation and random.random() < 0.5

    def _img(img):
        if hflip:
            img = img[:, ::-1, ...]
        if vflip:
            img = img[::-1, :, ...]
        if rot90:
            img = img.transpose(1, 0, 2) if img.ndim == 3 else img.T
        return np.ascontiguousarray(img)

    def _flow(flow):
        flow = flow.copy()
        if hflip:
            flow = flow[:, ::-1, :].copy()
            flow[:, :, 0] *= -1
        if vflip:
            flow = flow[::-1, :, :].copy()
            flow[:, :, 1] *= -1
        if rot90:
            flow = flow.transpose(1, 0, 2)[:, :, [1, 0]]
        return np.ascontiguousarray(flow)

    single = not isinstance(imgs, list)
    out = [_img(i) for i in ([imgs] if single else imgs)]
    out = out[0] if len(out) == 1 else out
    if flows is not None:
        fl = [_flow(f) for f in (flows if isinstance(flows, list) else [flows])]
        fl = fl[0] if len(fl) == 1 else fl
        return (out, fl, (hflip, vflip, rot90)) if return_status else (out, fl)
    return (out, (hflip, vflip, rot90)) if return_status else out
