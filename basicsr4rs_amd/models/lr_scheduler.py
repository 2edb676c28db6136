"""LR schedules used by the SR configs (basicsr/models/lr_scheduler.py:6-96)."""
import math
from collections import Counter

from torch.optim.lr_scheduler import _LRScheduler


class MultiStepRestartLR(_LRScheduler):
    """Step decay by ``gamma`` at each milestone; at a restart iteration the lr jumps back to
    ``initial_lr * restart_weight``."""

    def __init__(self, optimizer, milestones, gamma=0.1, restarts=(0, ), restart_weights=(1, ), last_epoch=-1):
        self.milestones = Counter(milestones)
        self.gamma = gamma
        self.restarts = restarts
        self.restart_weights = restart_weights
        assert len(self.restarts) == len(self.restart_weights), 'restarts and their weights do not match.'
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        groups = self.optimizer.param_groups
        if self.last_epoch in self.restarts:
            w = self.restart_weights[self.restarts.index(self.last_epoch)]
            return [g['initial_lr'] * w for g in groups]
        k = self.milestones.get(self.last_epoch, 0)
        return [g['lr'] * (self.gamma**k) for g in groups]


def get_position_from_periods(iteration, cumulative_period):
    """Index of the first cumulative period end >= iteration."""
    for i, end in enumerate(cumulative_period):
        if iteration <= end:
            return i


class CosineAnnealingRestartLR(_LRScheduler):
    """Cosine annealing over ``periods`` with weighted restarts, floor ``eta_min``."""

    def __init__(self, optimizer, periods, restart_weights=(1, ), eta_min=0, last_epoch=-1):
        self.periods = periods
        self.restart_weights = restart_weights
        self.eta_min = eta_min
        assert len(self.periods) == len(self.restart_weights), 'periods and restart_weights should have the same length.'
        self.cumulative_period = [sum(self.periods[:i + 1]) for i in range(len(self.periods))]
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        idx = get_position_from_periods(self.last_epoch, self.cumulative_period)
        w = self.restart_weights[idx]
        start = 0 if idx == 0 else self.cumulative_period[idx - 1]
        frac = (self.last_epoch - start) / self.periods[idx]
        return [self.eta_min + w * 0.5 * (b - self.eta_min) * (1 + math.cos(math.pi * frac)) for b in self.base_lrs]
