"""Loader-side prefetching (basicsr/data/prefetch_dataloader.py:8-122).

* PrefetchDataLoader: batches produced by a background thread into a bounded queue
  (num_prefetch_queue), so collation overlaps the train step.
* CPUPrefetcher: plain iterator wrapper with next() / reset().
* CUDAPrefetcher: the next batch's host->device copies run on a side HIP stream while the
  current step computes; ``next()`` makes the compute stream wait on that stream and marks the
  tensors as used by it (record_stream), so the caching allocator never hands their memory
  to another stream early.  Batches come from a pin_memory loader, so the copies are true
  async DMA transfers (pageable memory would serialise them behind a staging copy).
"""
import queue as Queue
import threading

import torch
from torch.utils.data import DataLoader


class PrefetchGenerator(threading.Thread):

    def __init__(self, generator, num_prefetch_queue):
        threading.Thread.__init__(self, daemon=True)
        self.queue = Queue.Queue(num_prefetch_queue)
        self.generator = generator
        self.start()

    def run(self):
        for item in self.generator:
            self.queue.put(item)
        self.queue.put(None)

    def __next__(self):
        item = self.queue.get()
        if item is None:
            raise StopIteration
        return item

    def __iter__(self):
        return self


class PrefetchDataLoader(DataLoader):

    def __init__(self, num_prefetch_queue, **kwargs):
        self.num_prefetch_queue = num_prefetch_queue
        super().__init__(**kwargs)

    def __iter__(self):
        return PrefetchGenerator(super().__iter__(), self.num_prefetch_queue)


class CPUPrefetcher:

    def __init__(self, loader):
        self.ori_loader = loader
        self.loader = iter(loader)

    def next(self):
        try:
            return next(self.loader)
        except StopIteration:
            return None

    def reset(self):
        self.loader = iter(self.ori_loader)


class CUDAPrefetcher:

    def __init__(self, loader, opt):
        self.ori_loader = loader
        self.loader = iter(loader)
        self.opt = opt
        self.stream = torch.cuda.Stream()
        self.device = torch.device('cuda' if opt.get('num_gpu', 1) != 0 else 'cpu')
        self.preload()

    def preload(self):
        try:
            self.batch = next(self.loader)
        except StopIteration:
            self.batch = None
            return
        with torch.cuda.stream(self.stream):
            for k, v in self.batch.items():
                if torch.is_tensor(v):
                    self.batch[k] = v.to(device=self.device, non_blocking=True)

    def next(self):
        cur = torch.cuda.current_stream()
        cur.wait_stream(self.stream)
        batch = self.batch
        if batch is not None:
            for v in batch.values():
                if torch.is_tensor(v) and v.is_cuda:
                    v.record_stream(cur)
        self.preload()
        return batch

    def reset(self):
        self.loader = iter(self.ori_loader)
        self.preload()
