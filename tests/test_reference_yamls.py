"""The reference's own hot-path option files (north_star: "options/train YAMLs ... still work"):
every EDSR / RCAN / SwinIR / RRDBNet-PSNR / MSRResNet train and test YAML of /root/reference is
read by this package's ``parse_options`` (basicsr/utils/options.py:99-201 contract) and its
``network_g`` built by ``build_network`` (basicsr/archs/__init__.py:18-24) with the reference's
kwargs; ``model_type``, the pixel loss, the scheduler and the optimizer must resolve to what this
package implements, and the datasets to registered types (or to the remote-sensing readers whose
packages the image lacks).  Container-only: skipped where /root/reference is absent
(the GPU box).  The YAMLs are read as data; no reference code is imported or run.

Not covered: ``train_SwinIR_StyleCNN_*.yml`` name ``SwinIR_StyleCNN``, an arch the reference itself
does not define (no ``class SwinIR_StyleCNN`` anywhere under basicsr/); ``train_SwinIR_L2S288_scratch.yml``
selects the Landsat-to-Sentinel family (``SwinIRL2sModel``, ``L2SSingleHMSplitDataset``,
basicsr/models/srrs_l2s_model.py), out of scope with the fork's remote-sensing data readers
(SURVEY.md §2)."""
import glob
import os

import pytest
import torch

REF = '/root/reference/options'
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason='reference option files not present')

PATTERNS = ['train/EDSR/*.yml', 'train/RCAN/*.yml', 'train/SwinIR/train_SwinIR_S[R2]*.yml',
            'train/ESRGAN/train_RRDBNet_PSNR_x4.yml', 'train/SRResNet_SRGAN/train_MSRResNet_x*.yml', 'test/EDSR/*.yml',
            'test/RCAN/*.yml', 'test/SwinIR/*.yml', 'test/ESRGAN/test_RRDBNet*.yml']
# dataset types of the fork whose readers need packages absent from this image (tacoreader, lmdb)
ABSENT_DATASETS = {'TacoSplitDataset'}
# (pattern, network type, params) spot checks against the reference nets' known sizes
SIZES = {'train/EDSR/train_EDSR_Lx4.yml': ('EDSR', 43089923), 'train/RCAN/train_RCAN_x2.yml': ('RCAN', 15444643),
         'train/ESRGAN/train_RRDBNet_PSNR_x4.yml': ('RRDBNet', 16697987)}


def _files():
    out = []
    for p in PATTERNS:
        out += sorted(glob.glob(os.path.join(REF, p)))
    return [os.path.relpath(f, REF) for f in out]


@pytest.mark.parametrize('rel', _files() if os.path.isdir(REF) else ['none'])
def test_reference_yaml_parses_and_builds(rel, tmp_path):
    import basicsr4rs_amd.archs  # noqa: F401
    import basicsr4rs_amd.data  # noqa: F401
    import basicsr4rs_amd.losses  # noqa: F401
    import basicsr4rs_amd.models  # noqa: F401
    from basicsr4rs_amd.archs import build_network
    from basicsr4rs_amd.models import lr_scheduler
    from basicsr4rs_amd.utils.options import parse_options
    from basicsr4rs_amd.utils.registry import DATASET_REGISTRY, LOSS_REGISTRY, MODEL_REGISTRY
    is_train = rel.startswith('train/')
    opt, _ = parse_options(str(tmp_path), is_train=is_train, argv=['-opt', os.path.join(REF, rel)])
    assert opt['model_type'] in MODEL_REGISTRY, opt['model_type']
    torch.manual_seed(0)
    net = build_network(dict(opt['network_g']))
    n = sum(p.numel() for p in net.parameters())
    if rel in SIZES:
        assert (type(net).__name__, n) == SIZES[rel]
    for phase, ds in opt.get('datasets', {}).items():
        assert ds['type'] in DATASET_REGISTRY or ds['type'] in ABSENT_DATASETS, (phase, ds['type'])
        assert ds['phase'] == phase.split('_')[0]
    if is_train:
        tr = opt['train']
        assert tr['pixel_opt']['type'] in LOSS_REGISTRY
        assert tr['optim_g']['type'] in ('Adam', 'AdamW')
        sched = tr['scheduler']['type']
        assert sched in ('MultiStepLR', 'MultiStepRestartLR', 'CosineAnnealingRestartLR'), sched
        assert hasattr(lr_scheduler, 'MultiStepRestartLR') and hasattr(lr_scheduler, 'CosineAnnealingRestartLR')
        assert opt['path']['models'].startswith(str(tmp_path))
