"""EnlargedSampler (basicsr/data/data_sampler.py:6-48): each rank takes indices
rank::world of an epoch-seeded permutation of an enlarged index range, so one "epoch" of
the loader covers ``ratio`` passes over the dataset (iteration-based training restarts the
loader less often)."""
import math

import torch
from torch.utils.data.sampler import Sampler


class EnlargedSampler(Sampler):

    def __init__(self, dataset, num_replicas, rank, ratio=1):
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.num_samples = math.ceil(len(self.dataset) * ratio / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def __iter__(self):
        g = torch.Generator()
        g.manual_seed(self.epoch)  # same permutation on every rank for an epoch
        perm = torch.randperm(self.total_size, generator=g)
        idx = (perm % len(self.dataset))[self.rank::self.num_replicas].tolist()
        assert len(idx) == self.num_samples
        return iter(idx)

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch):
        self.epoch = epoch
