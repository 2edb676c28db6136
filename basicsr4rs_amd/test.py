"""Test entry point (the contract of basicsr/test.py:11-45): ``python -m basicsr4rs_amd.test
-opt options/test/X.yml``: results dirs, one loader per test dataset, ``build_model`` with
``is_train=False`` and ``model.validation`` (metrics, optional SR image dump) on each."""
import logging
from os import path as osp

from .data import build_dataloader, build_dataset
from .models import build_model
from .utils.logger import get_env_info, get_root_logger
from .utils.misc import get_time_str, make_exp_dirs
from .utils.options import dict2str, parse_options

import basicsr4rs_amd.archs  # noqa: F401,E402  (registers the nets)


def test_pipeline(root_path, argv=None):
    opt, _ = parse_options(root_path, is_train=False, argv=argv)
    make_exp_dirs(opt)
    log_file = osp.join(opt['path']['log'], f"test_{opt['name']}_{get_time_str()}.log")
    logger = get_root_logger(logger_name='basicsr', log_level=logging.INFO, log_file=log_file)
    logger.info(get_env_info())
    logger.info(dict2str(opt))
    loaders = []
    for _, dataset_opt in sorted(opt['datasets'].items()):
        ds = build_dataset(dataset_opt)
        loaders.append(build_dataloader(ds, dataset_opt, num_gpu=opt['num_gpu'], dist=opt['dist'], sampler=None,
                                        seed=opt['manual_seed']))
        logger.info(f"Number of test images in {dataset_opt['name']}: {len(ds)}")
    model = build_model(opt)
    for loader in loaders:
        logger.info(f"Testing {loader.dataset.opt['name']}...")
        model.validation(loader, current_iter=opt['name'], tb_logger=None, save_img=opt['val']['save_img'])
    return model


if __name__ == '__main__':
    test_pipeline(osp.abspath(osp.join(__file__, osp.pardir, osp.pardir)))
