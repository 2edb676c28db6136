"""The train entry point on the HIP engine (basicsr/train.py:92-216 + options.py:99-201):
a YAML with the keys of options/train/EDSR/train_EDSR_Lx4.yml (small net and data, written by
the test) trains 3 iterations with checkpoint / validation cadence, then ``--auto_resume``
picks the newest training state and continues to iteration 5."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

YML = """
name: 206_EDSR_Lx4_tiny
model_type: SRModel
scale: 4
num_gpu: 1
manual_seed: 10
datasets:
  train:
    name: DIV2K
    type: PairedImageDataset
    dataroot_gt: {root}/gt
    dataroot_lq: {root}/lq
    filename_tmpl: '{{}}'
    io_backend:
      type: disk
    gt_size: 64
    use_hflip: true
    use_rot: true
    num_worker_per_gpu: 0
    batch_size_per_gpu: 2
    dataset_enlarge_ratio: 2
    prefetch_mode: ~
  val:
    name: Set5
    type: PairedImageDataset
    dataroot_gt: {root}/gt
    dataroot_lq: {root}/lq
    io_backend:
      type: disk
network_g:
  type: EDSR
  num_in_ch: 3
  num_out_ch: 3
  num_feat: 64
  num_block: 2
  upscale: 4
  res_scale: 0.1
  img_range: 255.
  rgb_mean: [0.4488, 0.4371, 0.4040]
path:
  pretrain_network_g: ~
  strict_load_g: true
  resume_state: ~
train:
  ema_decay: 0.999
  optim_g:
    type: Adam
    lr: !!float 1e-4
    weight_decay: 0
    betas: [0.9, 0.99]
  scheduler:
    type: MultiStepLR
    milestones: [200000]
    gamma: 0.5
  total_iter: 3
  warmup_iter: -1
  pixel_opt:
    type: L1Loss
    loss_weight: 1.0
    reduction: mean
val:
  val_freq: !!float 2
  save_img: true
  metrics:
    psnr:
      type: calculate_psnr
      crop_border: 4
      test_y_channel: false
logger:
  print_freq: 1
  save_checkpoint_freq: !!float 2
  use_tb_logger: false
  wandb:
    project: ~
    resume_id: ~
dist_params:
  backend: nccl
  port: 29500
"""


def test_train_pipeline_from_yaml_then_auto_resume(cuda, tmp_path):
    from basicsr4rs_amd.train import train_pipeline
    from basicsr4rs_amd.utils.logger import reset_root_logger
    from tests.test_data import _make_pairs
    _make_pairs(tmp_path, 4, 16, 16, 4)
    yml = tmp_path / 'train_EDSR_Lx4.yml'
    yml.write_text(YML.format(root=str(tmp_path)))
    root = str(tmp_path / 'run')
    os.makedirs(root)
    reset_root_logger()
    m1 = train_pipeline(root, argv=['-opt', str(yml)])
    exp = os.path.join(root, 'experiments', '206_EDSR_Lx4_tiny')
    for f in ('models/net_g_2.pth', 'models/net_g_latest.pth', 'training_states/2.state', 'train_EDSR_Lx4.yml'):
        assert os.path.isfile(os.path.join(exp, f)), f
    assert float(m1.optimizer_g.state_dict()['state'][0]['step']) == 3.0
    assert m1.metric_results['psnr'] > 0
    assert list((tmp_path / 'run' / 'experiments' / '206_EDSR_Lx4_tiny' / 'visualization').rglob('*_2.png'))
    ck = torch.load(os.path.join(exp, 'models', 'net_g_2.pth'), map_location='cpu', weights_only=True)
    assert set(ck) == {'params', 'params_ema'}
    logs = [f for f in os.listdir(exp) if f.startswith('train_') and f.endswith('.log')]
    log_text = open(os.path.join(exp, logs[0])).read()
    assert logs and 'l_pix:' in log_text
    # the validation metric record of basicsr/models/sr_model.py:252-266, with the best value
    assert 'Validation Set5' in log_text and '# psnr: ' in log_text and 'Best: ' in log_text

    # auto-resume from the newest state (iter 2) and run on to iteration 5
    reset_root_logger()
    m2 = train_pipeline(root, argv=['-opt', str(yml), '--auto_resume', '--force_yml', 'train:total_iter=5'])
    assert float(m2.optimizer_g.state_dict()['state'][0]['step']) == 5.0
    assert os.path.isfile(os.path.join(exp, 'training_states', '4.state'))
    assert m2.opt['path']['pretrain_network_g'] == os.path.join(exp, 'models', 'net_g_2.pth')
    logs = sorted(os.path.join(exp, f) for f in os.listdir(exp) if f.startswith('train_') and f.endswith('.log'))
    assert any('Resuming training from epoch: 0, iter: 2.' in open(f).read() for f in logs)
    reset_root_logger()
