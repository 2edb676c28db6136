"""Options: YAML -> OrderedDict, the train / test CLI, seeds and the experiment path layout
(the contract of basicsr/utils/options.py:13-219).

CLI: ``-opt X.yml --launcher {none,pytorch,slurm} --auto_resume --debug --local_rank N
--force_yml a:b=v ...``.  Differences from the reference, all on the safe side:
* the YAML is read with a SafeLoader subclass (mappings as OrderedDict) -- no python tags;
* ``--force_yml`` walks the key path instead of exec-ing a string, and a list value is parsed
  with ``ast.literal_eval`` instead of ``eval``; only existing keys may be set, as before;
* the process-group backend comes from ``dist_params.backend`` (default 'nccl' = RCCL),
  so a gloo rehearsal of the multi-process path is one YAML key.
"""
import argparse
import ast
import os
import random
import sys
import time
from collections import OrderedDict
from os import path as osp
from shutil import copyfile

import torch
import yaml

from .dist_util import get_dist_info, init_dist, master_only
from .misc import set_random_seed


class _OrderedSafeLoader(yaml.SafeLoader):
    pass


def _construct_mapping(loader, node):
    loader.flatten_mapping(node)
    return OrderedDict(loader.construct_pairs(node))


_OrderedSafeLoader.add_constructor(yaml.resolver.BaseResolver.DEFAULT_MAPPING_TAG, _construct_mapping)


class _OrderedDumper(yaml.SafeDumper):
    pass


_OrderedDumper.add_representer(OrderedDict, lambda d, data: d.represent_dict(data.items()))


def ordered_yaml():
    """(Loader, Dumper) keeping mapping order (options.py:13-35), safe variants."""
    return _OrderedSafeLoader, _OrderedDumper


def yaml_load(f):
    """Load a YAML file path or a YAML string."""
    if os.path.isfile(f):
        with open(f, 'r') as fh:
            return yaml.load(fh, Loader=_OrderedSafeLoader)
    return yaml.load(f, Loader=_OrderedSafeLoader)


def dict2str(opt, indent_level=1):
    msg = '\n'
    pad = ' ' * (indent_level * 2)
    for k, v in opt.items():
        if isinstance(v, dict):
            msg += f'{pad}{k}:[' + dict2str(v, indent_level + 1) + f'{pad}]\n'
        else:
            msg += f'{pad}{k}: {v}\n'
    return msg


def _postprocess_yml_value(value):
    """A --force_yml right-hand side -> None / bool / !!float / int / float / list / str."""
    if value == '~' or value.lower() == 'none':
        return None
    if value.lower() in ('true', 'false'):
        return value.lower() == 'true'
    if value.startswith('!!float'):
        return float(value.replace('!!float', ''))
    if value.isdigit():
        return int(value)
    if value.replace('.', '', 1).isdigit() and value.count('.') < 2:
        return float(value)
    if value.startswith('['):
        return ast.literal_eval(value)
    return value


def _force(opt, entry):
    keys, value = entry.split('=')
    path = [k for k in keys.strip().split(':')]
    node = opt
    for k in path[:-1]:
        node = node[k]
    if path[-1] not in node:  # as the reference: no new keys
        raise KeyError(f'--force_yml: {keys.strip()} is not an existing option')
    node[path[-1]] = _postprocess_yml_value(value.strip())


def parse_args(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument('-opt', type=str, required=True, help='Path to option YAML file.')
    parser.add_argument('--launcher', choices=['none', 'pytorch', 'slurm'], default='none', help='job launcher')
    parser.add_argument('--auto_resume', action='store_true')
    parser.add_argument('--debug', action='store_true')
    parser.add_argument('--local_rank', type=int, default=0)
    parser.add_argument('--force_yml', nargs='+', default=None,
                        help='Force to update yml files. Examples: train:ema_decay=0.999')
    return parser.parse_args(argv)


def parse_options(root_path, is_train=True, argv=None):
    """(opt, args) for the train / test pipelines; ``argv`` defaults to sys.argv[1:]."""
    args = parse_args(argv)
    opt = yaml_load(args.opt)

    if args.launcher == 'none':
        opt['dist'] = False
        print('Disable distributed.', flush=True)
    else:
        opt['dist'] = True
        dp = dict(opt.get('dist_params') or {})
        backend = dp.pop('backend', 'nccl')
        if args.launcher == 'slurm':
            init_dist('slurm', backend=backend)
        else:
            init_dist('pytorch', backend=backend)
    opt['rank'], opt['world_size'] = get_dist_info()

    seed = opt.get('manual_seed')
    if seed is None:
        seed = random.randint(1, 10000)
        opt['manual_seed'] = seed
    set_random_seed(seed + opt['rank'])

    for entry in args.force_yml or []:
        _force(opt, entry)

    opt['auto_resume'] = args.auto_resume
    opt['is_train'] = is_train
    if args.debug and not opt['name'].startswith('debug'):
        opt['name'] = 'debug_' + opt['name']
    if opt.get('num_gpu') == 'auto':
        opt['num_gpu'] = torch.cuda.device_count()

    for phase, dataset in opt.get('datasets', {}).items():
        dataset['phase'] = phase.split('_')[0]  # val_1, val_2 -> val
        if 'scale' in opt:
            dataset['scale'] = opt['scale']
        for key in ('dataroot_gt', 'dataroot_lq'):
            if dataset.get(key) is not None:
                dataset[key] = osp.expanduser(dataset[key])

    opt.setdefault('path', OrderedDict())
    for key, val in opt['path'].items():
        if val is not None and ('resume_state' in key or 'pretrain_network' in key):
            opt['path'][key] = osp.expanduser(val)

    if is_train:
        root = osp.join(opt['path'].get('experiments_root') or osp.join(root_path, 'experiments'), opt['name'])
        opt['path']['experiments_root'] = root
        opt['path']['models'] = osp.join(root, 'models')
        opt['path']['training_states'] = osp.join(root, 'training_states')
        opt['path']['log'] = root
        opt['path']['visualization'] = osp.join(root, 'visualization')
        if 'debug' in opt['name']:
            if 'val' in opt:
                opt['val']['val_freq'] = 8
            opt['logger']['print_freq'] = 1
            opt['logger']['save_checkpoint_freq'] = 8
    else:
        root = osp.join(opt['path'].get('results_root') or osp.join(root_path, 'results'), opt['name'])
        opt['path']['results_root'] = root
        opt['path']['log'] = root
        opt['path']['visualization'] = osp.join(root, 'visualization')
    return opt, args


@master_only
def copy_opt_file(opt_file, experiments_root):
    """Copy the YAML into the run directory with a generation-time / command header."""
    dst = osp.join(experiments_root, osp.basename(opt_file))
    copyfile(opt_file, dst)
    with open(dst, 'r+') as f:
        lines = f.readlines()
        lines.insert(0, f"# GENERATE TIME: {time.asctime()}\n# CMD:\n# {' '.join(sys.argv)}\n\n")
        f.seek(0)
        f.writelines(lines)
