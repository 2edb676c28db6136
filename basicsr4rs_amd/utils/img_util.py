"""Tensor <-> uint8 image helpers (mirror of basicsr/utils/img_util.py:40-96).

OpenCV is not available in this image: RGB->BGR is a channel flip and ``imwrite`` writes
PNG with the standard library (zlib) so validation images can still be saved.
"""
import math
import os
import struct
import zlib

import numpy as np
import torch


def make_grid(t, nrow=8, padding=2, pad_value=0.0, value_range=None):
    """torchvision.utils.make_grid for a [B, C, H, W] batch (the 4-D branch of tensor2img,
    img_util.py:72-76, and ``minusone_one_tensor_to_ubyte_numpy``): 1-channel maps repeated to 3,
    ``value_range=(lo, hi)`` = normalize=True over that range (clamp, then (x - lo) / (hi - lo)),
    a single image returned as is, else tiles on a pad_value canvas, ``nrow`` per row."""
    if t.size(1) == 1:
        t = torch.cat((t, t, t), 1)
    if value_range is not None:
        lo, hi = value_range
        t = t.clamp(min=lo, max=hi).sub(lo).div(max(hi - lo, 1e-5))
    if t.size(0) == 1:
        return t.squeeze(0)
    nmaps = t.size(0)
    xmaps = min(nrow, nmaps)
    ymaps = int(math.ceil(float(nmaps) / xmaps))
    height, width = int(t.size(2) + padding), int(t.size(3) + padding)
    grid = t.new_full((t.size(1), height * ymaps + padding, width * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= nmaps:
                break
            grid[:, y * height + padding:(y + 1) * height, x * width + padding:(x + 1) * width] = t[k]
            k += 1
    return grid


def tensor2img(tensor, rgb2bgr=True, out_type=np.uint8, min_max=(0, 1)):
    """Clamp to min_max, scale to [0,1], CHW->HWC, RGB->BGR, *255 and round for uint8
    (basicsr/utils/img_util.py:40-96; a 4-D batch is tiled with make_grid first)."""
    if not (torch.is_tensor(tensor) or (isinstance(tensor, list) and all(torch.is_tensor(t) for t in tensor))):
        raise TypeError(f'tensor or list of tensors expected, got {type(tensor)}')
    if torch.is_tensor(tensor):
        tensor = [tensor]
    result = []
    for t in tensor:
        t = t.squeeze(0).float().detach().cpu().clamp_(*min_max)
        t = (t - min_max[0]) / (min_max[1] - min_max[0])
        if t.dim() == 4:
            img = make_grid(t, nrow=int(math.sqrt(t.size(0)))).numpy().transpose(1, 2, 0)
            if rgb2bgr:
                img = img[..., ::-1]
        elif t.dim() == 3:
            img = t.numpy().transpose(1, 2, 0)
            if img.shape[2] == 1:
                img = np.squeeze(img, axis=2)
            elif rgb2bgr:
                img = img[..., ::-1]
        elif t.dim() == 2:
            img = t.numpy()
        else:
            raise TypeError(f'Only support 4D, 3D or 2D tensor. But received with dimension: {t.dim()}')
        if out_type == np.uint8:
            img = (img * 255.0).round()
        result.append(np.ascontiguousarray(img).astype(out_type))
    return result[0] if len(result) == 1 else result


def img_as_ubyte(img):
    """skimage.util.img_as_ubyte of a float image in [-1, 1] (the fork's conversion,
    basicsr/utils/img_util.py:8,128): x * 255 in the input's float type, round half to even, clip to
    [0, 255]; negative values clip to 0."""
    img = np.asarray(img)
    if img.dtype.kind != 'f':
        raise TypeError(f'img_as_ubyte: float image expected, got {img.dtype}')
    if img.size and (img.min() < -1.0 or img.max() > 1.0):
        raise ValueError('Images of type float must be between -1 and 1.')
    ct = np.float32 if img.dtype.itemsize <= 4 else img.dtype
    out = np.multiply(img, 255, dtype=ct)
    np.rint(out, out=out)
    np.clip(out, 0, 255, out=out)
    return out.astype(np.uint8)


def zero_one_tensor_to_ubyte_numpy(tensor):
    """A [B, C, H, W] tensor in [0, 1] -> one H x (B W) x C uint8 image (basicsr/utils/img_util.py:
    115-128): the batch tiled in one row by make_grid (2-px zero padding when B > 1, normalized over
    (0, 1)), channel order kept (no RGB -> BGR flip), then img_as_ubyte."""
    t = tensor.detach().float().cpu()
    grid = make_grid(t, nrow=t.size(0), value_range=(0, 1))
    return img_as_ubyte(grid.numpy().transpose(1, 2, 0))


def minusone_one_tensor_to_ubyte_numpy(tensor):
    """The fork's remote-sensing image conversion (basicsr/utils/img_util.py:99-112): a [B, C, H, W]
    tensor in [-1, 1] is clamped to [-1, 1], mapped to (x + 1) / 2 and converted as
    ``zero_one_tensor_to_ubyte_numpy``."""
    t = torch.clamp(tensor.detach().float().cpu(), -1, 1)
    return zero_one_tensor_to_ubyte_numpy((t + 1) / 2)


def imwrite(img, file_path, params=None, auto_mkdir=True):
    """Write a uint8 HWC BGR (or HW gray) image as PNG."""
    if auto_mkdir:
        os.makedirs(os.path.dirname(os.path.abspath(file_path)), exist_ok=True)
    img = np.asarray(img, dtype=np.uint8)
    if img.ndim == 3:
        img = img[..., ::-1]  # BGR -> RGB for PNG
        h, w, c = img.shape
        ctype = {3: 2, 4: 6, 1: 0}[c]
    else:
        h, w = img.shape
        c, ctype = 1, 0
    raw = b''.join(b'\x00' + img[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xffffffff)

    png = b'\x89PNG\r\n\x1a\n' + chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, 8, ctype, 0, 0, 0))
    png += chunk(b'IDAT', zlib.compress(raw, 6)) + chunk(b'IEND', b'')
    with open(file_path, 'wb') as f:
        f.write(png)
    return True


def imfrombytes(content, flag='color', float32=False):
    """Decode image bytes to a numpy HWC BGR array (basicsr/utils/img_util.py:99-117 semantics:
    ``color`` -> 3-channel BGR, ``grayscale`` -> HW, ``unchanged`` keeps depth / alpha;
    ``float32`` divides by 255).  Decoded with Pillow (OpenCV is not in this image); ``.npy``
    payloads (HWC arrays, no pickle) are accepted as well."""
    import io
    if content[:6] == b'\x93NUMPY':
        img = np.load(io.BytesIO(content), allow_pickle=False)
    else:
        from PIL import Image
        with Image.open(io.BytesIO(content)) as im:
            if flag == 'grayscale':
                img = np.asarray(im.convert('L'))
            elif flag == 'color':
                img = np.asarray(im.convert('RGB'))[..., ::-1]
            else:
                img = np.asarray(im)
                if img.ndim == 3 and img.shape[2] in (3, 4):
                    img = img[..., [2, 1, 0] + ([3] if img.shape[2] == 4 else [])]
    img = np.ascontiguousarray(img)
    if float32:
        img = img.astype(np.float32) / 255.
    return img


def img2tensor(imgs, bgr2rgb=True, float32=True):
    """Numpy HWC -> tensor CHW (basicsr/utils/img_util.py:11-37), BGR -> RGB for 3 channels."""

    def _one(img):
        if img.ndim == 2:
            img = img[..., None]
        if img.shape[2] == 3 and bgr2rgb:
            img = img[..., ::-1]
        t = torch.from_numpy(np.ascontiguousarray(img.transpose(2, 0, 1)))
        return t.float() if float32 else t

    return [_one(i) for i in imgs] if isinstance(imgs, list) else _one(imgs)


def scandir(dir_path, suffix=None, recursive=False, full_path=False):
    """Sorted-walk file scan relative to ``dir_path`` (basicsr/utils/misc.py:57-91)."""
    if suffix is not None and not isinstance(suffix, (str, tuple)):
        raise TypeError('"suffix" must be a string or tuple of strings')
    root = dir_path

    def _scan(path):
        for entry in sorted(os.scandir(path), key=lambda e: e.name):
            if not entry.name.startswith('.') and entry.is_file():
                rel = entry.path if full_path else os.path.relpath(entry.path, root)
                if suffix is None or rel.endswith(suffix):
                    yield rel
            elif recursive and entry.is_dir():
                yield from _scan(entry.path)

    return _scan(dir_path)
