"""LR schedules (basicsr/models/lr_scheduler.py:6-96) on a CPU dummy optimizer."""
import math

import torch

from basicsr4rs_amd.models.lr_scheduler import CosineAnnealingRestartLR, MultiStepRestartLR


def _opt(lr=1.0):
    return torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=lr)


def test_multistep_restart():
    o = _opt()
    s = MultiStepRestartLR(o, milestones=[2, 4], gamma=0.5, restarts=[0, 5], restart_weights=[1, 0.1])
    lrs = []
    for _ in range(7):
        lrs.append(o.param_groups[0]['lr'])
        o.step()
        s.step()
    assert lrs == [1.0, 1.0, 0.5, 0.5, 0.25, 0.1, 0.1]


def test_cosine_restart():
    o = _opt()
    s = CosineAnnealingRestartLR(o, periods=[4, 4], restart_weights=[1, 0.5], eta_min=0.0)
    lrs = []
    for _ in range(8):
        lrs.append(o.param_groups[0]['lr'])
        o.step()
        s.step()
    assert abs(lrs[2] - 0.5 * (1 + math.cos(math.pi * 2 / 4))) < 1e-9
    assert abs(lrs[5] - 0.5 * 0.5 * (1 + math.cos(math.pi * 1 / 4))) < 1e-9
