"""Validation metrics and image conversion on the host (basicsr/metrics/psnr_ssim.py,
basicsr/metrics/metric_util.py, basicsr/utils/img_util.py:40-96).

Pinned by the reference's own metric tests (tests/test_metrics/test_psnr_ssim.py: shape
assert, input-order ValueError, float result, PSNR(identical) = inf) plus closed-form
known answers.  The reference's SSIM filters with OpenCV, which is absent here: the numpy
form is checked against an independent direct 2-D valid correlation (scipy) and against the
tensor form, so SSIM parity with cv2 itself is "parity unpinned" beyond these identities."""
import numpy as np
import pytest
import torch

from basicsr4rs_amd.metrics import calculate_metric, calculate_psnr, calculate_psnr_pt, calculate_ssim, calculate_ssim_pt
from basicsr4rs_amd.metrics.psnr_ssim import _to_y, gaussian_window
from basicsr4rs_amd.utils.img_util import make_grid, tensor2img


def test_reference_psnr_contract():
    with pytest.raises(AssertionError):
        calculate_psnr(np.ones((16, 16)), np.ones((10, 10)), crop_border=0)
    with pytest.raises(ValueError):
        calculate_psnr(np.ones((16, 16)), np.ones((16, 16)), crop_border=1, input_order='WRONG')
    out = calculate_psnr(np.ones((10, 10, 3)), np.ones((10, 10, 3)) * 2, crop_border=1, test_y_channel=True)
    assert isinstance(out, float)
    assert calculate_psnr(np.ones((10, 10, 3)), np.ones((10, 10, 3)), crop_border=0) == float('inf')


def test_reference_ssim_contract():
    with pytest.raises(AssertionError):
        calculate_ssim(np.ones((16, 16)), np.ones((10, 10)), crop_border=0)
    with pytest.raises(ValueError):
        calculate_ssim(np.ones((16, 16)), np.ones((16, 16)), crop_border=1, input_order='WRONG')
    out = calculate_ssim(np.ones((10, 10, 3)), np.ones((10, 10, 3)) * 2, crop_border=1, test_y_channel=True)
    assert isinstance(out, float)


def test_to_y_channel_known_answers():
    """metric_util.to_y_channel: 3-channel BGR -> 16 + (24.966 B + 128.553 G + 65.481 R) / 255
    in [0,255]; a 1-channel image is returned unchanged (x / 255 * 255)."""
    img = np.zeros((2, 2, 3), dtype=np.uint8)
    img[0, 0] = (255, 255, 255)
    img[0, 1] = (255, 0, 0)  # blue only
    y = _to_y(img)
    assert y.shape == (2, 2, 1)
    assert abs(y[0, 0, 0] - (16 + 219.0)) < 1e-3
    assert abs(y[0, 1, 0] - (16 + 24.966)) < 1e-3
    assert abs(y[1, 1, 0] - 16.0) < 1e-4
    gray = np.array([[0, 128], [200, 255]], dtype=np.uint8)[..., None]
    assert np.allclose(_to_y(gray), gray.astype(np.float32), atol=1e-4)
    # grayscale PSNR with test_y_channel equals the plain PSNR (the round-1 1/255 bug is gone)
    g2 = gray.copy()
    g2[0, 0] = 3
    assert abs(calculate_psnr(gray, g2, 0, test_y_channel=True) - calculate_psnr(gray, g2, 0)) < 1e-6


def test_gaussian_window_matches_closed_form():
    w = gaussian_window()
    x = np.arange(11) - 5.0
    k = np.exp(-x**2 / 4.5)
    assert np.allclose(w, np.outer(k, k) / k.sum()**2, atol=1e-15)
    assert abs(w.sum() - 1.0) < 1e-12 and w.shape == (11, 11)


def _ssim_direct(a, b):
    """Independent restatement with scipy's 2-D valid correlation (psnr_ssim.py:261-276)."""
    from scipy.signal import correlate2d
    w = gaussian_window()
    f = lambda t: correlate2d(t, w, mode='valid')  # noqa: E731
    c1, c2 = (0.01 * 255)**2, (0.03 * 255)**2
    mu1, mu2 = f(a), f(b)
    s1, s2, s12 = f(a * a) - mu1**2, f(b * b) - mu2**2, f(a * b) - mu1 * mu2
    return (((2 * mu1 * mu2 + c1) * (2 * s12 + c2)) / ((mu1**2 + mu2**2 + c1) * (s1 + s2 + c2))).mean()


def _pair(seed=0, shape=(40, 36, 3)):
    rs = np.random.RandomState(seed)
    a = rs.randint(0, 256, shape).astype(np.uint8)
    b = np.clip(a.astype(int) + rs.randint(-12, 13, shape), 0, 255).astype(np.uint8)
    return a, b


def test_ssim_matches_direct_correlation_and_identities():
    a, b = _pair()
    ref = np.mean([_ssim_direct(a[..., c].astype(np.float64), b[..., c].astype(np.float64)) for c in range(3)])
    assert abs(calculate_ssim(a, b, crop_border=0) - ref) < 1e-12
    assert calculate_ssim(a, a, crop_border=4) == pytest.approx(1.0, abs=1e-12)
    assert calculate_ssim(a, b, crop_border=0) < 1.0
    # CHW order and crop
    assert abs(calculate_ssim(a.transpose(2, 0, 1), b.transpose(2, 0, 1), 3, input_order='CHW') -
               calculate_ssim(a, b, 3)) < 1e-12


@pytest.mark.parametrize('y', [False, True])
def test_tensor_metrics_match_numpy(y):
    """calculate_psnr_pt / calculate_ssim_pt on [0,1] RGB tensors equal the numpy metrics on the
    same images as uint8 BGR (tensor2img), per image (psnr_ssim.py:91-121, :210-245)."""
    imgs = [_pair(s) for s in (1, 2)]
    ta = torch.stack([torch.from_numpy(a[..., ::-1].copy()).permute(2, 0, 1) for a, _ in imgs]).double() / 255.
    tb = torch.stack([torch.from_numpy(b[..., ::-1].copy()).permute(2, 0, 1) for _, b in imgs]).double() / 255.
    p = calculate_psnr_pt(ta, tb, crop_border=2, test_y_channel=y)
    s = calculate_ssim_pt(ta, tb, crop_border=2, test_y_channel=y)
    assert p.shape == (2, ) and s.shape == (2, )
    for i, (a, b) in enumerate(imgs):
        assert tensor2img(ta[i]).tolist() == a.tolist()
        # psnr_pt adds 1e-8 to the [0,1] MSE (psnr_ssim.py:121): ~6e-5 dB here
        assert abs(p[i].item() - calculate_psnr(a, b, 2, test_y_channel=y)) < 1e-3
        assert abs(s[i].item() - calculate_ssim(a, b, 2, test_y_channel=y)) < (1e-4 if y else 1e-9)


def test_tensor2img_contract():
    t = torch.tensor([[[0.0, 0.5], [1.2, -0.1]], [[0.25, 0.75], [0.1, 0.9]], [[1.0, 0.0], [0.5, 0.5]]])
    img = tensor2img(t)
    assert img.dtype == np.uint8 and img.shape == (2, 2, 3)
    # RGB -> BGR, clamp to [0,1], x255, round
    assert img[0, 0].tolist() == [255, 64, 0]
    assert img[1, 0].tolist() == [128, 26, 255]
    assert img[1, 1].tolist() == [128, 230, 0]
    assert tensor2img(t, rgb2bgr=False)[0, 0].tolist() == [0, 64, 255]
    f = tensor2img(t, out_type=np.float32)
    assert f.dtype == np.float32 and abs(f[0, 1, 2] - 0.5) < 1e-7
    # [-1, 1] range, gray and 2-D inputs, batch dim 1 squeezed, list input
    assert tensor2img(torch.zeros(1, 1, 3, 3), min_max=(-1, 1)).tolist() == [[128] * 3] * 3
    assert tensor2img(torch.ones(3, 4)).shape == (3, 4)
    assert len(tensor2img([t, t])) == 2
    with pytest.raises(TypeError):
        tensor2img(np.zeros((2, 2)))
    # 4-D batch: make_grid tiles (nrow = floor(sqrt(B))), padding 2
    b = torch.rand(4, 3, 5, 6)
    g = tensor2img(b, rgb2bgr=False)
    assert g.shape == (2 * 7 + 2, 2 * 8 + 2, 3)
    assert np.array_equal(g[2:7, 10:16], (b[1].permute(1, 2, 0).numpy() * 255).round().astype(np.uint8))
    assert make_grid(b, nrow=2).shape == (3, 16, 18)


def test_metric_registry_dispatch():
    a, b = _pair(3)
    v = calculate_metric(dict(img=a, img2=b), dict(type='calculate_ssim', crop_border=4, test_y_channel=True))
    assert abs(v - calculate_ssim(a, b, 4, test_y_channel=True)) < 1e-12
    v = calculate_metric(dict(img=a, img2=b), dict(type='calculate_psnr', crop_border=4, test_y_channel=False))
    assert abs(v - calculate_psnr(a, b, 4)) < 1e-12


def test_minusone_one_to_ubyte_matches_oracle():
    """The fork's [-1, 1] -> uint8 conversion (basicsr/utils/img_util.py:99-128: clamp, (x + 1) / 2,
    make_grid normalize over (0, 1), img_as_ubyte) against the numpy restatement in
    oracle/metrics.py, bit-exact: 4-band and 1-band images, one image and a padded batch row,
    values outside [-1, 1]; known answers -1 -> 0, 0 -> 128 (127.5 rounds half to even), 1 -> 255."""
    import numpy as np
    import torch

    from basicsr4rs_amd.utils.img_util import minusone_one_tensor_to_ubyte_numpy
    from oracle import metrics as OM
    g = torch.Generator().manual_seed(5)
    for shape in ((1, 4, 9, 7), (3, 4, 5, 6), (1, 1, 4, 4), (2, 1, 3, 5), (2, 3, 4, 4)):
        t = torch.rand(shape, generator=g) * 3 - 1.5
        got = minusone_one_tensor_to_ubyte_numpy(t)
        ref = OM.minusone_one_to_ubyte(t.numpy())
        assert got.dtype == np.uint8 and got.shape == ref.shape, (shape, got.shape, ref.shape)
        assert np.array_equal(got, ref), shape
    k = minusone_one_tensor_to_ubyte_numpy(torch.tensor([-1.0, 0.0, 1.0, -7.0]).view(1, 1, 1, 4))
    assert k[0, :, 0].tolist() == [0, 128, 255, 0]
    assert minusone_one_tensor_to_ubyte_numpy(torch.zeros(2, 4, 3, 3)).shape == (3 + 4, 2 * (3 + 2) + 2, 4)
