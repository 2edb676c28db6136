"""Run-directory, seeding and resume helpers of the train entry point (the contract of
basicsr/utils/misc.py:11-125): seeds, timestamped names, experiment dir layout, and the
resume rule that re-points ``pretrain_network_*`` at the checkpoint of the resumed iteration."""
import os
import random
import time
from os import path as osp

import numpy as np
import torch

from .dist_util import master_only
from .img_util import scandir

__all__ = ['set_random_seed', 'get_time_str', 'mkdir_and_rename', 'make_exp_dirs', 'check_resume', 'scandir']


def set_random_seed(seed):
    """Seed python, numpy and torch (CPU and every visible device) with one value (misc.py:11-17)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def get_time_str():
    return time.strftime('%Y%m%d_%H%M%S', time.localtime())


def mkdir_and_rename(path):
    """Create ``path``; an existing directory is first moved aside as ``<path>_archived_<time>``."""
    if osp.exists(path):
        archived = f'{path}_archived_{get_time_str()}'
        print(f'Path already exists. Rename it to {archived}', flush=True)
        os.rename(path, archived)
    os.makedirs(path, exist_ok=True)


@master_only
def make_exp_dirs(opt):
    """experiments_root (or results_root) fresh, then every other path entry that names a dir."""
    paths = dict(opt['path'])
    mkdir_and_rename(paths.pop('experiments_root' if opt['is_train'] else 'results_root'))
    skip = ('strict_load', 'pretrain_network', 'resume', 'param_key')
    for key, p in paths.items():
        if p is None or any(s in key for s in skip):
            continue
        os.makedirs(p, exist_ok=True)


def check_resume(opt, resume_iter):
    """On resume, load every ``network_*`` from ``models/net_<name>_<iter>.pth`` (unless listed in
    ``path.ignore_resume_networks``) and read the plain 'params' key of those checkpoints."""
    if not opt['path'].get('resume_state'):
        return
    networks = [k for k in opt if k.startswith('network_')]
    if any(opt['path'].get(f'pretrain_{n}') is not None for n in networks):
        print('pretrain_network path will be ignored during resuming.')
    ignore = opt['path'].get('ignore_resume_networks') or []
    for n in networks:
        if n in ignore:
            continue
        key = f'pretrain_{n}'
        opt['path'][key] = osp.join(opt['path']['models'], f"net_{n[len('network_'):]}_{resume_iter}.pth")
        print(f"Set {key} to {opt['path'][key]}")
    for key in [k for k in opt['path'] if k.startswith('param_key')]:
        if opt['path'][key] == 'params_ema':
            opt['path'][key] = 'params'
            print(f'Set {key} to params')
