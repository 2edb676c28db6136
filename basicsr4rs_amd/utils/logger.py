"""Console / file logging of the train loop (the contract of basicsr/utils/logger.py:10-185).

``get_root_logger``: rank 0 logs at INFO (plus a file handler when given), other ranks only
errors.  ``MessageLogger`` formats the per-``print_freq`` line (epoch, iter, lr, eta,
iter / data time, losses).  ``AvgTimer`` is the windowed wall-clock average the loop uses.
Tensorboard / wandb are optional: neither package is in this image, so ``init_tb_logger``
returns None with a warning instead of failing the run.
"""
import datetime
import logging
import time

from .dist_util import get_dist_info, master_only

_INITIALIZED = set()


class AvgTimer:
    """Mean of the intervals between consecutive ``record`` calls, restarted every ``window``."""

    def __init__(self, window=200):
        self.window = window
        self.current_time = 0.0
        self.total_time = 0.0
        self.count = 0
        self.avg_time = 0.0
        self.start()

    def start(self):
        self.start_time = self.tic = time.time()

    def record(self):
        self.count += 1
        self.toc = time.time()
        self.current_time = self.toc - self.tic
        self.total_time += self.current_time
        self.avg_time = self.total_time / self.count
        if self.count > self.window:
            self.count, self.total_time = 0, 0.0
        self.tic = time.time()

    def get_current_time(self):
        return self.current_time

    def get_avg_time(self):
        return self.avg_time


def get_root_logger(logger_name='basicsr', log_level=logging.INFO, log_file=None):
    logger = logging.getLogger(logger_name)
    if logger_name in _INITIALIZED:
        return logger
    fmt = logging.Formatter('%(asctime)s %(levelname)s: %(message)s')
    sh = logging.StreamHandler()
    sh.setFormatter(fmt)
    logger.addHandler(sh)
    logger.propagate = False
    if get_dist_info()[0] != 0:
        logger.setLevel('ERROR')
    else:
        logger.setLevel(log_level)
        if log_file is not None:
            fh = logging.FileHandler(log_file, 'w')
            fh.setFormatter(fmt)
            fh.setLevel(log_level)
            logger.addHandler(fh)
    _INITIALIZED.add(logger_name)
    return logger


def reset_root_logger(logger_name='basicsr'):
    """Drop the handlers of a logger so the next get_root_logger re-initialises it (one process
    running several train pipelines, e.g. a run and its auto-resume in the tests)."""
    logger = logging.getLogger(logger_name)
    for h in list(logger.handlers):
        logger.removeHandler(h)
        h.close()
    _INITIALIZED.discard(logger_name)


class MessageLogger:
    """Formats one log line per ``print_freq`` iterations (logger.py:45-115)."""

    def __init__(self, opt, start_iter=1, tb_logger=None):
        self.exp_name = opt['name']
        self.interval = opt['logger']['print_freq']
        self.start_iter = start_iter
        self.max_iters = opt['train']['total_iter']
        self.use_tb_logger = opt['logger'].get('use_tb_logger', False)
        self.tb_logger = tb_logger
        self.start_time = time.time()
        self.logger = get_root_logger()

    def reset_start_time(self):
        self.start_time = time.time()

    @master_only
    def __call__(self, log_vars):
        log_vars = dict(log_vars)
        epoch, current_iter, lrs = log_vars.pop('epoch'), log_vars.pop('iter'), log_vars.pop('lrs')
        msg = f'[{self.exp_name[:5]}..][epoch:{epoch:3d}, iter:{current_iter:8,d}, lr:('
        msg += ''.join(f'{v:.3e},' for v in lrs) + ')] '
        if 'time' in log_vars:
            iter_time, data_time = log_vars.pop('time'), log_vars.pop('data_time')
            per_iter = (time.time() - self.start_time) / (current_iter - self.start_iter + 1)
            eta = str(datetime.timedelta(seconds=int(per_iter * (self.max_iters - current_iter - 1))))
            msg += f'[eta: {eta}, time (data): {iter_time:.3f} ({data_time:.3f})] '
        for k, v in log_vars.items():
            msg += f'{k}: {v:.4e} '
            if self.tb_logger is not None and 'debug' not in self.exp_name:
                self.tb_logger.add_scalar(f'losses/{k}' if k.startswith('l_') else k, v, current_iter)
        self.logger.info(msg)


@master_only
def init_tb_logger(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
    except ImportError:
        get_root_logger().warning('tensorboard is not installed: use_tb_logger ignored')
        return None
    return SummaryWriter(log_dir=log_dir)


def get_env_info():
    import torch
    from .. import _lib
    try:
        hip = _lib.load().sr_version().decode()
    except ImportError as e:  # the run fails at the first HIP op anyway; report it here first
        hip = f'not built ({e})'
    return (f'\nVersion Information:\n\tbasicsr4rs_amd (libsr_hip): {hip}\n\tPyTorch: {torch.__version__}'
            f"\n\tHIP: {getattr(torch.version, 'hip', None)}")
