"""Input pipeline (basicsr/data/*): EnlargedSampler, paired crop / augment,
PairedImageDataset over image folders, build_dataloader with seeded workers and the CPU
prefetch queue.  CPU only; the CUDA prefetcher is in test_data_gpu below (marked gpu)."""
import math
import random

import numpy as np
import pytest
import torch

from basicsr4rs_amd.data import EnlargedSampler, build_dataloader, build_dataset
from basicsr4rs_amd.data.transforms import augment, mod_crop, paired_random_crop
from basicsr4rs_amd.utils.img_util import imfrombytes, imwrite


class _Len:

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


def _reference_indices(n, world, rank, ratio, epoch):
    """The reference algorithm written out (data_sampler.py:29-42)."""
    num_samples = math.ceil(n * ratio / world)
    total = num_samples * world
    g = torch.Generator()
    g.manual_seed(epoch)
    idx = [v % n for v in torch.randperm(total, generator=g).tolist()]
    return idx[rank:total:world]


@pytest.mark.parametrize('n,world,ratio', [(10, 1, 1), (10, 3, 1), (7, 4, 100), (1, 2, 3)])
def test_enlarged_sampler(n, world, ratio):
    for epoch in (0, 5):
        parts = []
        for rank in range(world):
            s = EnlargedSampler(_Len(n), world, rank, ratio)
            s.set_epoch(epoch)
            got = list(iter(s))
            assert got == _reference_indices(n, world, rank, ratio, epoch)
            assert len(got) == len(s) == math.ceil(n * ratio / world)
            parts.append(got)
        # ranks partition the enlarged range: every index appears ratio (or ceil) times overall
        counts = np.bincount(np.concatenate(parts), minlength=n)
        assert counts.min() >= (n * ratio) // n and counts.sum() == len(parts[0]) * world
    a = EnlargedSampler(_Len(50), 1, 0)
    b = EnlargedSampler(_Len(50), 1, 0)
    b.set_epoch(1)
    assert list(a) != list(b)


def test_paired_random_crop_aligned():
    rng = np.random.default_rng(0)
    lq = rng.random((20, 24, 3)).astype(np.float32)
    gt = np.repeat(np.repeat(lq, 4, 0), 4, 1)  # exact x4 nearest upsample: crops must line up
    random.seed(1)
    for _ in range(10):
        g, l = paired_random_crop(gt, lq, 32, 4)
        assert g.shape == (32, 32, 3) and l.shape == (8, 8, 3)
        assert np.array_equal(g[::4, ::4], l)
    with pytest.raises(ValueError):
        paired_random_crop(gt[:-1], lq, 32, 4)
    with pytest.raises(ValueError):
        paired_random_crop(gt, lq, 256, 4)
    t_g, t_l = paired_random_crop(torch.tensor(gt.transpose(2, 0, 1)), torch.tensor(lq.transpose(2, 0, 1)), 16, 4)
    assert t_g.shape == (3, 16, 16) and torch.equal(t_g[:, ::4, ::4], t_l)
    assert mod_crop(np.zeros((10, 11, 3)), 4).shape == (8, 8, 3)


def test_augment_pairs_identically():
    rng = np.random.default_rng(1)
    lq = rng.random((6, 6, 3)).astype(np.float32)
    gt = np.repeat(np.repeat(lq, 2, 0), 2, 1)
    seen = set()
    random.seed(3)
    for _ in range(40):
        (g, l), st = augment([gt, lq], True, True, return_status=True)
        seen.add(st)
        assert np.array_equal(g[::2, ::2], l)
        ref = lq
        if st[0]:
            ref = ref[:, ::-1]
        if st[1]:
            ref = ref[::-1]
        if st[2]:
            ref = ref.transpose(1, 0, 2)
        assert np.array_equal(l, ref)
    assert len(seen) == 8  # every flip / rotation combination occurs
    flow = rng.random((6, 6, 2)).astype(np.float32)
    random.seed(0)
    _, f2, st = augment(lq, True, True, flows=flow, return_status=True)
    assert f2.shape == flow.shape


def _make_pairs(tmp_path, n, h, w, scale):
    rng = np.random.default_rng(2)
    (tmp_path / 'lq').mkdir()
    (tmp_path / 'gt').mkdir()
    for i in range(n):
        lq = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        gt = np.repeat(np.repeat(lq, scale, 0), scale, 1)
        imwrite(lq, str(tmp_path / 'lq' / f'{i:04d}.png'))
        imwrite(gt, str(tmp_path / 'gt' / f'{i:04d}.png'))


def test_imfrombytes_roundtrip(tmp_path):
    img = np.random.default_rng(5).integers(0, 256, (5, 7, 3), dtype=np.uint8)
    imwrite(img, str(tmp_path / 'a.png'))
    got = imfrombytes(open(tmp_path / 'a.png', 'rb').read())
    assert np.array_equal(got, img)  # BGR in, BGR out
    assert np.allclose(imfrombytes(open(tmp_path / 'a.png', 'rb').read(), float32=True), img / 255.)


def test_paired_dataset_and_loader(tmp_path):
    _make_pairs(tmp_path, 6, 16, 20, 4)
    opt = dict(name='t', type='PairedImageDataset', dataroot_gt=str(tmp_path / 'gt'), dataroot_lq=str(tmp_path / 'lq'),
               io_backend=dict(type='disk'), gt_size=32, use_hflip=True, use_rot=True, scale=4, phase='train',
               batch_size_per_gpu=2, num_worker_per_gpu=2)
    ds = build_dataset(opt)
    assert len(ds) == 6
    item = ds[0]
    assert item['lq'].shape == (3, 8, 8) and item['gt'].shape == (3, 32, 32)
    assert torch.equal(item['gt'][:, ::4, ::4], item['lq'])
    assert item['lq'].dtype == torch.float32 and 0 <= item['lq'].min() and item['lq'].max() <= 1
    sampler = EnlargedSampler(ds, 1, 0, ratio=2)
    for mode in (None, 'cpu'):
        o = dict(opt, prefetch_mode=mode)
        loader = build_dataloader(ds, o, num_gpu=1, dist=False, sampler=sampler, seed=10)
        batches = list(loader)
        assert len(batches) == 6  # 12 enlarged samples / batch 2
        assert batches[0]['lq'].shape == (2, 3, 8, 8) and batches[0]['gt'].shape == (2, 3, 32, 32)
        for b in batches:
            assert torch.equal(b['gt'][..., ::4, ::4], b['lq'])
    # seeded workers: the same crops twice
    l1 = [b['lq'] for b in build_dataloader(ds, opt, sampler=sampler, seed=10)]
    l2 = [b['lq'] for b in build_dataloader(ds, opt, sampler=sampler, seed=10)]
    assert all(torch.equal(a, b) for a, b in zip(l1, l2))
    # val phase: full images, GT cropped to scale * LQ, RGB order
    v = build_dataset(dict(opt, phase='val'))[1]
    assert v['lq'].shape == (3, 16, 20) and v['gt'].shape == (3, 64, 80)
    raw = imfrombytes(open(v['lq_path'], 'rb').read(), float32=True)
    assert torch.allclose(v['lq'], torch.tensor(raw[..., ::-1].copy()).permute(2, 0, 1))


@pytest.mark.gpu
def test_cuda_prefetcher_feeds_model_buffers(cuda, tmp_path):
    from basicsr4rs_amd.data import CUDAPrefetcher
    _make_pairs(tmp_path, 4, 16, 16, 2)
    opt = dict(name='t', type='PairedImageDataset', dataroot_gt=str(tmp_path / 'gt'), dataroot_lq=str(tmp_path / 'lq'),
               io_backend=dict(type='disk'), gt_size=16, use_hflip=False, use_rot=False, scale=2, phase='train',
               batch_size_per_gpu=2, num_worker_per_gpu=0, pin_memory=True)
    ds = build_dataset(opt)
    loader = build_dataloader(ds, opt, sampler=EnlargedSampler(ds, 1, 0), seed=0)
    pf = CUDAPrefetcher(loader, dict(num_gpu=1))
    n = 0
    b = pf.next()
    while b is not None:
        assert b['lq'].is_cuda and b['gt'].shape == (2, 3, 16, 16)
        assert torch.equal(b['gt'][..., ::2, ::2], b['lq'])
        n += 1
        b = pf.next()
    assert n == 2
    pf.reset()
    assert pf.next() is not None


def test_prefetch_loader_and_cpu_prefetcher():
    """PrefetchDataLoader yields the DataLoader's batches in order, stays exhausted, and re-raises
    a loading error in the consumer; CPUPrefetcher returns None at the end of an epoch and
    restarts on reset() (basicsr/data/prefetch_dataloader.py API, basicsr/train.py:170-209 loop)."""
    from basicsr4rs_amd.data.prefetch_dataloader import CPUPrefetcher, PrefetchDataLoader
    data = torch.arange(10.).view(10, 1)
    loader = PrefetchDataLoader(num_prefetch_queue=2, dataset=data, batch_size=3)
    it = iter(loader)
    got = list(it)
    assert [b.tolist() for b in got] == [b.tolist() for b in torch.utils.data.DataLoader(data, batch_size=3)]
    with pytest.raises(StopIteration):
        next(it)

    class Bad(torch.utils.data.Dataset):
        def __len__(self):
            return 4

        def __getitem__(self, i):
            if i == 2:
                raise ValueError('corrupt sample 2')
            return torch.tensor([float(i)])

    with pytest.raises(ValueError, match='corrupt sample 2'):
        list(PrefetchDataLoader(num_prefetch_queue=1, dataset=Bad(), batch_size=1))
    # a caller that catches and continues gets the error again, not a blocked queue
    bad_it = iter(PrefetchDataLoader(num_prefetch_queue=1, dataset=Bad(), batch_size=1))
    assert next(bad_it).item() == 0 and next(bad_it).item() == 1
    for _ in range(2):
        with pytest.raises(ValueError, match='corrupt sample 2'):
            next(bad_it)
    pf = CPUPrefetcher(torch.utils.data.DataLoader(data, batch_size=5))
    assert pf.next().shape == (5, 1) and pf.next() is not None and pf.next() is None
    pf.reset()
    assert torch.equal(pf.next(), data[:5])
