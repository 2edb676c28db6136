"""Loader-side prefetching: the API of basicsr/data/prefetch_dataloader.py (PrefetchDataLoader,
CPUPrefetcher, CUDAPrefetcher with ``next()`` / ``reset()``), built around one staging idea.

* ``PrefetchDataLoader(num_prefetch_queue, **loader_kwargs)``: iterating it runs the DataLoader
  iterator on a background thread that keeps up to ``num_prefetch_queue`` collated batches in a
  bounded queue, so collation overlaps the train step.  Unlike a bare producer thread, an
  exception raised while loading is carried through the queue and re-raised in the consumer
  (the step loop sees the real error instead of hanging or stopping early).
* ``CPUPrefetcher``: batches as the loader yields them.
* ``CUDAPrefetcher``: the next batch's host->device copies are queued on a side HIP stream while
  the current step computes; handing a batch out makes the compute stream wait on that stream and
  records the tensors as used by it (``record_stream``), so the caching allocator never gives
  their memory to another stream early.  With a pin_memory loader the copies are true async DMA.

Both prefetchers share ``_Prefetcher``: it holds one staged batch ahead (``_stage``) and returns
None once the epoch is exhausted, which is how the train loop (basicsr/train.py:170-209) detects
the end of an epoch.
"""
import queue
import threading

import torch
from torch.utils.data import DataLoader

_END = object()


class _LoaderError:
    __slots__ = ('exc', )

    def __init__(self, exc):
        self.exc = exc


class _QueuedIterator:
    """Drains ``source`` on a daemon thread into a queue of at most ``depth`` items."""

    def __init__(self, source, depth):
        self._q = queue.Queue(maxsize=max(1, int(depth)))
        self._thread = threading.Thread(target=self._fill, args=(source, ), daemon=True)
        self._thread.start()

    def _fill(self, source):
        try:
            for item in source:
                self._q.put(item)
        except BaseException as exc:  # surfaced in the consumer thread
            self._q.put(_LoaderError(exc))
            return
        self._q.put(_END)

    def __iter__(self):
        return self

    def __next__(self):
        item = self._q.get()
        if item is _END:
            self._q.put(_END)  # stay exhausted on repeated next()
            raise StopIteration
        if isinstance(item, _LoaderError):
            self._q.put(item)  # the producer is gone: a repeated next() raises again instead of blocking
            raise item.exc
        return item


class PrefetchDataLoader(DataLoader):
    """A DataLoader whose iterator is read ahead by a background thread (num_prefetch_queue)."""

    def __init__(self, num_prefetch_queue, **kwargs):
        self.num_prefetch_queue = num_prefetch_queue
        super().__init__(**kwargs)

    def __iter__(self):
        return _QueuedIterator(super().__iter__(), self.num_prefetch_queue)


class _Prefetcher:
    """One batch staged ahead of the consumer; ``next()`` returns None at the end of an epoch."""

    def __init__(self, loader):
        self.ori_loader = loader
        self._it = iter(loader)
        self._staged = None

    def _stage(self, batch):
        return batch

    def _pull(self):
        try:
            return next(self._it)
        except StopIteration:
            return None

    def next(self):
        batch = self._pull()
        return None if batch is None else self._stage(batch)

    def reset(self):
        self._it = iter(self.ori_loader)


class CPUPrefetcher(_Prefetcher):
    """Batches as the loader yields them (basicsr/data/prefetch_dataloader.py:55-79 API)."""


class CUDAPrefetcher(_Prefetcher):
    """Side-stream host->device staging of the next batch (the reference's CUDAPrefetcher API)."""

    def __init__(self, loader, opt):
        super().__init__(loader)
        self.opt = opt
        self.device = torch.device('cuda' if opt.get('num_gpu', 1) != 0 else 'cpu')
        self.stream = torch.cuda.Stream()
        self._ahead = self._copy_next()

    def _copy_next(self):
        batch = self._pull()
        if batch is None:
            return None
        with torch.cuda.stream(self.stream):
            return {k: (v.to(device=self.device, non_blocking=True) if torch.is_tensor(v) else v)
                    for k, v in batch.items()}

    def next(self):
        batch = self._ahead
        compute = torch.cuda.current_stream()
        compute.wait_stream(self.stream)
        if batch is not None:
            for v in batch.values():
                if torch.is_tensor(v) and v.is_cuda:
                    v.record_stream(compute)
        self._ahead = self._copy_next()
        return batch

    def reset(self):
        super().reset()
        self._ahead = self._copy_next()
