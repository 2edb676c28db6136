"""Fixture: a real-image LR tile from the reference's own test data.

Reads /root/reference/test_scripts/data/baboon.png (492 x 480 RGB, the reference repository's
test image) with Pillow, takes the HR crop rows 160..415, cols 120..375 (256 x 256: fur and
eye, a wide range of values and edges), makes the x4 LR tile by 4x4 box averaging (64 x 64) and
stores both as uint8 HWC in tests/golden/baboon_x4.npz.  The tile is data, not reference code;
the GPU parity test feeds it to EDSR_M / RCAN / SwinIR against the CPU oracle
(tests/test_real_image_gpu.py), so the mean-shift / img_range 255 path sees real-image statistics
instead of U[0,1) noise.  Run once in the container (the reference does not travel)."""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    img = np.asarray(Image.open('/root/reference/test_scripts/data/baboon.png').convert('RGB'))
    hr = np.ascontiguousarray(img[160:416, 120:376])
    lr = hr.reshape(64, 4, 64, 4, 3).astype(np.float64).mean(axis=(1, 3))
    lr = np.clip(np.rint(lr), 0, 255).astype(np.uint8)
    np.savez_compressed(os.path.join(HERE, 'baboon_x4.npz'), hr=hr, lr=lr)
    print('hr', hr.shape, hr.mean(), 'lr', lr.shape, lr.mean())


if __name__ == '__main__':
    main()
