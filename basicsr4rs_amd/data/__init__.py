"""Datasets and loaders (basicsr/data/__init__.py:25-100): DATASET_REGISTRY auto-import of
``*_dataset.py`` modules, ``build_dataset``, ``build_dataloader`` (per-GPU batch / workers,
EnlargedSampler, seeded workers, optional CPU prefetch queue)."""
import importlib
import os.path as osp
import random
from copy import deepcopy
from functools import partial

import numpy as np
import torch
import torch.utils.data

from ..utils.dist_util import get_dist_info
from ..utils.img_util import scandir
from ..utils.registry import DATASET_REGISTRY
from .data_sampler import EnlargedSampler
from .prefetch_dataloader import CPUPrefetcher, CUDAPrefetcher, PrefetchDataLoader

__all__ = ['build_dataset', 'build_dataloader', 'EnlargedSampler', 'CPUPrefetcher', 'CUDAPrefetcher']

_folder = osp.dirname(osp.abspath(__file__))
_modules = [importlib.import_module(f'{__name__}.{osp.splitext(f)[0]}') for f in scandir(_folder)
            if f.endswith('_dataset.py')]


def build_dataset(dataset_opt):
    dataset_opt = deepcopy(dataset_opt)
    return DATASET_REGISTRY.get(dataset_opt['type'])(dataset_opt)


def worker_init_fn(worker_id, num_workers, rank, seed):
    """Worker seed = num_workers * rank + worker_id + seed (basicsr/data/__init__.py:96-100);
    Python ``random`` drives the crops, so it is seeded too."""
    s = num_workers * rank + worker_id + seed
    np.random.seed(s)
    random.seed(s)


def build_dataloader(dataset, dataset_opt, num_gpu=1, dist=False, sampler=None, seed=None):
    phase = dataset_opt['phase']
    rank, _ = get_dist_info()
    if phase == 'train':
        if dist:
            batch_size = dataset_opt['batch_size_per_gpu']
            num_workers = dataset_opt['num_worker_per_gpu']
        else:
            mult = 1 if num_gpu == 0 else num_gpu
            batch_size = dataset_opt['batch_size_per_gpu'] * mult
            num_workers = dataset_opt['num_worker_per_gpu'] * mult
        args = dict(dataset=dataset, batch_size=batch_size, shuffle=sampler is None, num_workers=num_workers,
                    sampler=sampler, drop_last=True)
        args['worker_init_fn'] = (partial(worker_init_fn, num_workers=num_workers, rank=rank, seed=seed)
                                  if seed is not None else None)
    elif phase in ('val', 'test'):
        args = dict(dataset=dataset, batch_size=1, shuffle=False, num_workers=0)
    else:
        raise ValueError(f"Wrong dataset phase: {phase}. Supported ones are 'train', 'val' and 'test'.")
    args['pin_memory'] = dataset_opt.get('pin_memory', False) and torch.cuda.is_available()
    args['persistent_workers'] = dataset_opt.get('persistent_workers', False) and args['num_workers'] > 0
    if dataset_opt.get('prefetch_mode') == 'cpu':
        return PrefetchDataLoader(num_prefetch_queue=dataset_opt.get('num_prefetch_queue', 1), **args)
    return torch.utils.data.DataLoader(**args)
