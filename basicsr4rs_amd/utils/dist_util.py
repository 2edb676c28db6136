"""Process-group helpers (mirror of basicsr/utils/dist_util.py:10-80).

One process per GPU; ``init_dist('pytorch')`` reads the torchrun environment
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), binds the process to its GPU and initialises
``torch.distributed`` with backend 'nccl' (= RCCL over xGMI on ROCm) or 'gloo' (CPU tests).
"""
import functools
import os

import torch
import torch.distributed as dist


def init_dist(launcher, backend='nccl', **kwargs):
    if launcher == 'pytorch':
        local = int(os.environ.get('LOCAL_RANK', os.environ.get('RANK', 0)))
        if backend == 'nccl':
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend, **kwargs)
    elif launcher == 'slurm':
        proc_id = int(os.environ['SLURM_PROCID'])
        ntasks = int(os.environ['SLURM_NTASKS'])
        ngpu = max(1, torch.cuda.device_count())
        os.environ.setdefault('MASTER_PORT', '29500')
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ['WORLD_SIZE'] = str(ntasks)
        os.environ['LOCAL_RANK'] = str(proc_id % ngpu)
        os.environ['RANK'] = str(proc_id)
        if backend == 'nccl':
            torch.cuda.set_device(proc_id % ngpu)
        dist.init_process_group(backend=backend)
    else:
        raise ValueError(f'Invalid launcher type: {launcher}')


def get_dist_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def master_only(func):

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        if get_dist_info()[0] == 0:
            return func(*args, **kwargs)

    return wrapper
