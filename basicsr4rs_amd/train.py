"""Train entry point (the contract of basicsr/train.py:17-216): ``python -m basicsr4rs_amd.train
-opt options/train/EDSR/train_EDSR_Lx4.yml [--launcher pytorch] [--auto_resume] [--debug]``.

Same flow as the reference loop: parse options (seed + rank, dist init), auto-resume from the
newest ``training_states/<iter>.state``, experiment dirs, train / val loaders over the
EnlargedSampler, ``build_model`` from MODEL_REGISTRY, then per iteration
``update_learning_rate -> feed_data -> optimize_parameters`` with logging every
``print_freq``, checkpoints every ``save_checkpoint_freq`` and validation every ``val_freq``;
the latest model is saved and validated at the end.  The step itself is the HIP engine's
(models/sr_model.py).  Under torchrun one process drives one GPU (RCCL gradient all-reduce).
"""
import datetime
import logging
import math
import time
from os import path as osp

import torch

from .data import build_dataloader, build_dataset
from .data.data_sampler import EnlargedSampler
from .data.prefetch_dataloader import CPUPrefetcher, CUDAPrefetcher
from .models import build_model
from .utils.logger import AvgTimer, MessageLogger, get_env_info, get_root_logger, init_tb_logger
from .utils.misc import check_resume, get_time_str, make_exp_dirs, mkdir_and_rename, scandir
from .utils.options import copy_opt_file, dict2str, parse_options

import basicsr4rs_amd.archs  # noqa: F401,E402  (registers the nets)


def init_tb_loggers(opt):
    if opt['logger'].get('use_tb_logger') and 'debug' not in opt['name']:
        return init_tb_logger(log_dir=osp.join(opt['root_path'], 'tb_logger', opt['name']))
    return None


def create_train_val_dataloader(opt, logger):
    train_loader, train_sampler, val_loaders = None, None, []
    total_epochs = total_iters = 0
    for phase, dataset_opt in opt['datasets'].items():
        if phase == 'train':
            ratio = dataset_opt.get('dataset_enlarge_ratio', 1)
            train_set = build_dataset(dataset_opt)
            train_sampler = EnlargedSampler(train_set, opt['world_size'], opt['rank'], ratio)
            train_loader = build_dataloader(train_set, dataset_opt, num_gpu=opt['num_gpu'], dist=opt['dist'],
                                            sampler=train_sampler, seed=opt['manual_seed'])
            iters_per_epoch = math.ceil(len(train_set) * ratio / (dataset_opt['batch_size_per_gpu'] * opt['world_size']))
            total_iters = int(opt['train']['total_iter'])
            total_epochs = math.ceil(total_iters / iters_per_epoch)
            logger.info(f'Training statistics:\n\tNumber of train images: {len(train_set)}'
                        f'\n\tDataset enlarge ratio: {ratio}\n\tBatch size per gpu: {dataset_opt["batch_size_per_gpu"]}'
                        f'\n\tWorld size (gpu number): {opt["world_size"]}\n\tRequire iter number per epoch: '
                        f'{iters_per_epoch}\n\tTotal epochs: {total_epochs}; iters: {total_iters}.')
        elif phase.split('_')[0] == 'val':
            val_set = build_dataset(dataset_opt)
            val_loaders.append(build_dataloader(val_set, dataset_opt, num_gpu=opt['num_gpu'], dist=opt['dist'],
                                                sampler=None, seed=opt['manual_seed']))
            logger.info(f'Number of val images/folders in {dataset_opt["name"]}: {len(val_set)}')
        else:
            raise ValueError(f'Dataset phase {phase} is not recognized.')
    return train_loader, train_sampler, val_loaders, total_epochs, total_iters


def load_resume_state(opt):
    """The newest training state under ``path.training_states`` with --auto_resume, else
    ``path.resume_state``; loaded tensors-only (weights_only) onto this process's device."""
    path = None
    if opt['auto_resume']:
        state_dir = opt['path']['training_states']
        if osp.isdir(state_dir):
            states = [float(v.split('.state')[0]) for v in scandir(state_dir, suffix='state')]
            if states:
                path = osp.join(state_dir, f'{max(states):.0f}.state')
                opt['path']['resume_state'] = path
    elif opt['path'].get('resume_state'):
        path = opt['path']['resume_state']
    if path is None:
        return None
    dev = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() else 'cpu'
    state = torch.load(path, map_location=dev, weights_only=True)
    check_resume(opt, state['iter'])
    return state


def train_pipeline(root_path, argv=None):
    opt, args = parse_options(root_path, is_train=True, argv=argv)
    opt['root_path'] = root_path

    resume_state = load_resume_state(opt)
    if resume_state is None:
        make_exp_dirs(opt)
        if opt['logger'].get('use_tb_logger') and 'debug' not in opt['name'] and opt['rank'] == 0:
            mkdir_and_rename(osp.join(root_path, 'tb_logger', opt['name']))
    copy_opt_file(args.opt, opt['path']['experiments_root'])

    log_file = osp.join(opt['path']['log'], f"train_{opt['name']}_{get_time_str()}.log")
    logger = get_root_logger(logger_name='basicsr', log_level=logging.INFO, log_file=log_file)
    logger.info(get_env_info())
    logger.info(dict2str(opt))
    tb_logger = init_tb_loggers(opt)

    train_loader, train_sampler, val_loaders, total_epochs, total_iters = create_train_val_dataloader(opt, logger)

    model = build_model(opt)
    if resume_state:
        model.resume_training(resume_state)
        logger.info(f"Resuming training from epoch: {resume_state['epoch']}, iter: {resume_state['iter']}.")
        start_epoch, current_iter = resume_state['epoch'], resume_state['iter']
    else:
        start_epoch, current_iter = 0, 0

    msg_logger = MessageLogger(opt, current_iter, tb_logger)
    prefetch_mode = opt['datasets']['train'].get('prefetch_mode')
    if prefetch_mode is None or prefetch_mode == 'cpu':
        prefetcher = CPUPrefetcher(train_loader)
    elif prefetch_mode == 'cuda':
        prefetcher = CUDAPrefetcher(train_loader, opt)
        logger.info(f'Use {prefetch_mode} prefetch dataloader')
        if opt['datasets']['train'].get('pin_memory') is not True:
            raise ValueError('Please set pin_memory=True for CUDAPrefetcher.')
    else:
        raise ValueError(f"Wrong prefetch_mode {prefetch_mode}. Supported ones are: None, 'cuda', 'cpu'.")

    logger.info(f'Start training from epoch: {start_epoch}, iter: {current_iter}')
    data_timer, iter_timer = AvgTimer(), AvgTimer()
    start_time = time.time()
    val_opt = opt.get('val')
    for epoch in range(start_epoch, total_epochs + 1):
        train_sampler.set_epoch(epoch)
        prefetcher.reset()
        train_data = prefetcher.next()
        while train_data is not None:
            data_timer.record()
            current_iter += 1
            if current_iter > total_iters:
                break
            model.update_learning_rate(current_iter, warmup_iter=opt['train'].get('warmup_iter', -1))
            model.feed_data(train_data)
            model.optimize_parameters(current_iter)
            iter_timer.record()
            if current_iter == 1:
                msg_logger.reset_start_time()
            if current_iter % opt['logger']['print_freq'] == 0:
                log_vars = {'epoch': epoch, 'iter': current_iter, 'lrs': model.get_current_learning_rate(),
                            'time': iter_timer.get_avg_time(), 'data_time': data_timer.get_avg_time()}
                log_vars.update(model.get_current_log())
                msg_logger(log_vars)
            if current_iter % opt['logger']['save_checkpoint_freq'] == 0:
                logger.info('Saving models and training states.')
                model.save(epoch, current_iter)
            if val_opt is not None and current_iter % val_opt['val_freq'] == 0:
                if len(val_loaders) > 1:
                    logger.warning('Multiple validation datasets are *only* supported by SRModel.')
                for val_loader in val_loaders:
                    model.validation(val_loader, current_iter, tb_logger, val_opt['save_img'])
            data_timer.start()
            iter_timer.start()
            train_data = prefetcher.next()

    logger.info(f'End of training. Time consumed: {datetime.timedelta(seconds=int(time.time() - start_time))}')
    logger.info('Save the latest model.')
    model.save(epoch=-1, current_iter=-1)
    if val_opt is not None:
        for val_loader in val_loaders:
            model.validation(val_loader, current_iter, tb_logger, val_opt['save_img'])
    if tb_logger:
        tb_logger.close()
    return model


if __name__ == '__main__':
    train_pipeline(osp.abspath(osp.join(__file__, osp.pardir, osp.pardir)))
