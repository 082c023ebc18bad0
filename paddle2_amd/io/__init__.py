"""paddle.io: Dataset / Sampler / DataLoader (reference: python/paddle/io/, dataloader_iter.py).

Workers (``num_workers > 0``) are separate processes that hand batches back through shared
memory (torch's multiprocessing machinery over /dev/shm, like the reference's
``_use_shared_memory``); the main process wraps them as Paddle Tensors on the current place,
copying from pinned memory asynchronously when the target is the MI355X.
"""
from __future__ import annotations

import bisect
import math
import numbers

import numpy as np
import torch

from ..framework.tensor import Tensor


class Dataset:
    def __getitem__(self, idx):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError


class IterableDataset(Dataset):
    def __iter__(self):
        raise NotImplementedError


class TensorDataset(Dataset):
    def __init__(self, tensors):
        self.tensors = tensors
        n = tensors[0].shape[0]
        assert all(t.shape[0] == n for t in tensors)

    def __getitem__(self, idx):
        return tuple(t[idx] for t in self.tensors)

    def __len__(self):
        return self.tensors[0].shape[0]


class ComposeDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, idx):
        out = []
        for d in self.datasets:
            s = d[idx]
            out.extend(s if isinstance(s, (list, tuple)) else [s])
        return tuple(out)


class ChainDataset(IterableDataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __iter__(self):
        for d in self.datasets:
            yield from d


class ConcatDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)
        self.cum = list(np.cumsum([len(d) for d in self.datasets]))

    def __len__(self):
        return self.cum[-1]

    def __getitem__(self, idx):
        if idx < 0:
            idx += len(self)
        di = bisect.bisect_right(self.cum, idx)
        base = 0 if di == 0 else self.cum[di - 1]
        return self.datasets[di][idx - base]


class Subset(Dataset):
    def __init__(self, dataset, indices):
        self.dataset, self.indices = dataset, list(indices)

    def __getitem__(self, idx):
        return self.dataset[self.indices[idx]]

    def __len__(self):
        return len(self.indices)


def random_split(dataset, lengths, generator=None):
    n = len(dataset)
    if all(isinstance(l, float) for l in lengths) and abs(sum(lengths) - 1) < 1e-6:
        lengths = [int(math.floor(n * f)) for f in lengths]
        for i in range(n - sum(lengths)):
            lengths[i % len(lengths)] += 1
    perm = np.random.permutation(n).tolist()
    out, off = [], 0
    for l in lengths:
        out.append(Subset(dataset, perm[off:off + l]))
        off += l
    return out


# ---------------------------------------------------------------------- samplers
class Sampler:
    def __init__(self, data_source=None):
        self.data_source = data_source

    def __iter__(self):
        raise NotImplementedError


class SequenceSampler(Sampler):
    def __iter__(self):
        return iter(range(len(self.data_source)))

    def __len__(self):
        return len(self.data_source)


class RandomSampler(Sampler):
    def __init__(self, data_source, replacement=False, num_samples=None, generator=None):
        super().__init__(data_source)
        self.replacement = replacement
        self._num = num_samples
        self.generator = generator

    @property
    def num_samples(self):
        return self._num if self._num is not None else len(self.data_source)

    def __iter__(self):
        n = len(self.data_source)
        if self.replacement:
            return iter(np.random.randint(0, n, self.num_samples).tolist())
        return iter(np.random.permutation(n)[: self.num_samples].tolist())

    def __len__(self):
        return self.num_samples


class SubsetRandomSampler(Sampler):
    def __init__(self, indices, generator=None):
        self.indices = list(indices)

    def __iter__(self):
        return iter([self.indices[i] for i in np.random.permutation(len(self.indices))])

    def __len__(self):
        return len(self.indices)


class WeightedRandomSampler(Sampler):
    def __init__(self, weights, num_samples, replacement=True):
        self.weights = np.asarray(weights._t.cpu() if isinstance(weights, Tensor) else weights, dtype=np.float64)
        self.num_samples, self.replacement = num_samples, replacement

    def __iter__(self):
        p = self.weights / self.weights.sum()
        return iter(np.random.choice(len(p), self.num_samples, replace=self.replacement, p=p).tolist())

    def __len__(self):
        return self.num_samples


class BatchSampler(Sampler):
    def __init__(self, dataset=None, sampler=None, shuffle=False, batch_size=1, drop_last=False):
        if sampler is None:
            sampler = RandomSampler(dataset) if shuffle else SequenceSampler(dataset)
        self.sampler, self.batch_size, self.drop_last = sampler, batch_size, drop_last

    def __iter__(self):
        batch = []
        for i in self.sampler:
            batch.append(i)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size


class DistributedBatchSampler(BatchSampler):
    """Shards the index space across data-parallel ranks (reference: io/dataloader/batch_sampler.py)."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False, drop_last=False):
        from ..distributed import collective as C

        self.dataset, self.batch_size, self.shuffle, self.drop_last = dataset, batch_size, shuffle, drop_last
        self.nranks = num_replicas if num_replicas is not None else C.get_world_size()
        self.local_rank = rank if rank is not None else C.get_rank()
        self.epoch = 0
        self.num_samples = int(math.ceil(len(dataset) * 1.0 / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def __iter__(self):
        n = len(self.dataset)
        idx = np.arange(n).tolist()
        idx += idx[: self.total_size - len(idx)]
        if self.shuffle:
            rs = np.random.RandomState(self.epoch)
            rs.shuffle(idx)
            self.epoch += 1
        # batch-strided subsample: rank r takes every nranks-th block of batch_size indices, and an
        # equal slice of the ragged tail (same assignment as the reference sampler)
        bs, nr, r = self.batch_size, self.nranks, self.local_rank
        tail = self.total_size % (bs * nr)
        mine = []
        for i in range(r * bs, len(idx) - tail, bs * nr):
            mine.extend(idx[i:i + bs])
        lt = tail // nr
        rest = idx[len(idx) - tail:]
        mine.extend(rest[r * lt:(r + 1) * lt])
        idx = mine
        batch = []
        for i in idx:
            batch.append(i)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = self.num_samples
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def set_epoch(self, epoch):
        self.epoch = epoch


# ---------------------------------------------------------------------- collate / loader
def _to_np(x):
    if isinstance(x, Tensor):
        return x.numpy()
    if isinstance(x, torch.Tensor):
        return x.numpy()
    return x


def default_collate_fn(batch):
    """Stacks samples field-wise into numpy arrays (numeric leaves) like paddle's collate."""
    sample = batch[0]
    if isinstance(sample, (np.ndarray, Tensor, torch.Tensor)):
        return np.stack([_to_np(b) for b in batch])
    if isinstance(sample, numbers.Number):
        return np.asarray(batch)
    if isinstance(sample, (str, bytes)):
        return list(batch)
    if isinstance(sample, dict):
        return {k: default_collate_fn([b[k] for b in batch]) for k in sample}
    if isinstance(sample, (list, tuple)):
        return [default_collate_fn(list(f)) for f in zip(*batch)]
    return batch


def default_convert_fn(batch):
    return batch


def _wrap_batch(obj, device, non_blocking):
    if isinstance(obj, np.ndarray):
        t = torch.from_numpy(obj) if obj.dtype != np.uint16 else torch.from_numpy(obj.view(np.int16)).view(torch.bfloat16)
        if obj.dtype == np.float64:
            t = t.float()
        return Tensor._wrap(t.to(device, non_blocking=non_blocking))
    if isinstance(obj, torch.Tensor):
        return Tensor._wrap(obj.to(device, non_blocking=non_blocking))
    if isinstance(obj, dict):
        return {k: _wrap_batch(v, device, non_blocking) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_wrap_batch(v, device, non_blocking) for v in obj]
    return obj


def _np_to_torch(obj):
    """Runs inside workers: numpy -> torch CPU tensors so the batch travels through shared memory."""
    if isinstance(obj, np.ndarray):
        if obj.dtype == np.uint16:
            return torch.from_numpy(np.ascontiguousarray(obj).view(np.int16)).view(torch.bfloat16)
        if obj.dtype == np.float64:
            return torch.from_numpy(obj.astype(np.float32))
        return torch.from_numpy(np.ascontiguousarray(obj))
    if isinstance(obj, dict):
        return {k: _np_to_torch(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_np_to_torch(v) for v in obj]
    return obj


class _TorchDatasetAdapter(torch.utils.data.Dataset):
    def __init__(self, ds):
        self.ds = ds

    def __getitem__(self, i):
        return self.ds[i]

    def __len__(self):
        return len(self.ds)


class _TorchIterAdapter(torch.utils.data.IterableDataset):
    def __init__(self, ds):
        self.ds = ds

    def __iter__(self):
        return iter(self.ds)


class _Collate:
    def __init__(self, fn):
        self.fn = fn or default_collate_fn

    def __call__(self, batch):
        return _np_to_torch(self.fn(batch))


class DataLoader:
    def __init__(self, dataset, feed_list=None, places=None, return_list=True, batch_sampler=None, batch_size=1,
                 shuffle=False, drop_last=False, collate_fn=None, num_workers=0, use_buffer_reader=True,
                 prefetch_factor=2, use_shared_memory=True, timeout=0, worker_init_fn=None, persistent_workers=False):
        self.dataset = dataset
        self.return_list = return_list
        self._use_buffer_reader = use_buffer_reader
        self._buffer_size = max(2, prefetch_factor)
        self.collate_fn = collate_fn
        self.num_workers = num_workers
        self.batch_size = batch_size
        is_iter = isinstance(dataset, IterableDataset)
        if batch_sampler is None and not is_iter:
            batch_sampler = BatchSampler(dataset, shuffle=shuffle, batch_size=batch_size, drop_last=drop_last)
        self.batch_sampler = batch_sampler
        from ..framework.place import _parse_device, current_torch_device

        self._device = _parse_device(places[0] if isinstance(places, (list, tuple)) else places) if places is not None \
            else current_torch_device()
        kw = dict(num_workers=num_workers, collate_fn=_Collate(collate_fn), timeout=timeout,
                  worker_init_fn=worker_init_fn, pin_memory=self._device.type == "cuda" and use_buffer_reader,
                  persistent_workers=persistent_workers and num_workers > 0)
        if num_workers > 0:
            kw["prefetch_factor"] = prefetch_factor
        if is_iter:
            self._loader = torch.utils.data.DataLoader(_TorchIterAdapter(dataset), batch_size=batch_size,
                                                       drop_last=drop_last, **kw)
        else:
            self._loader = torch.utils.data.DataLoader(_TorchDatasetAdapter(dataset), batch_sampler=batch_sampler, **kw)

    def __len__(self):
        return len(self.batch_sampler) if self.batch_sampler is not None else len(self._loader)

    def __iter__(self):
        nb = self._device.type == "cuda"
        if not self._use_buffer_reader:
            for batch in self._loader:
                yield _wrap_batch(batch, self._device, nb)
            return
        yield from _BufferedReader(self._loader, self._device, nb, self._buffer_size)

    def __call__(self):
        return self.__iter__()

    @staticmethod
    def from_generator(feed_list=None, capacity=None, use_double_buffer=True, iterable=True, return_list=False,
                       use_multiprocess=False, drop_last=True):
        return _GeneratorLoader()


class _BufferedReader:
    """Double-buffered reader (reference: LoDTensorBlockingQueue + BufferedReader, io/dataloader/
    dataloader_iter.py:154): a producer thread drains the sampler/worker pipeline, moves each batch
    to the device with non-blocking copies from pinned memory, and pushes it into the NATIVE bounded
    blocking queue (csrc/runtime/py_runtime.cpp BlockingQueue, waits with the GIL released); the
    training loop pops ready batches, so host collation and H2D copies overlap compute."""

    _END = ("__paddle2_amd_end__",)

    def __init__(self, loader, device, non_blocking, capacity):
        from .. import _rt

        self._q = _rt.get().BlockingQueue(capacity)
        self._err = None

        def produce():
            from ..profiler import host_range

            try:
                for batch in loader:
                    with host_range("DataLoader.prefetch", 3):
                        out = _wrap_batch(batch, device, non_blocking)
                    if not self._q.push(out):
                        return
            except BaseException as e:  # surfaced in the consumer
                self._err = e
            finally:
                self._q.push(self._END, 5.0)

        import threading

        self._th = threading.Thread(target=produce, daemon=True, name="pd-buffered-reader")
        self._th.start()

    def __iter__(self):
        try:
            while True:
                item = self._q.pop()
                if item is self._END:
                    break
                yield item
            if self._err is not None:
                raise self._err
        finally:
            self._q.close()


class _GeneratorLoader:
    def __init__(self):
        self._gen = None

    def set_batch_generator(self, reader, places=None):
        self._gen = reader

    def set_sample_list_generator(self, reader, places=None):
        self._gen = lambda: ([np.stack([s[i] for s in b]) for i in range(len(b[0]))] for b in reader())

    def __iter__(self):
        from ..framework.place import current_torch_device

        for b in self._gen():
            yield _wrap_batch(list(b) if isinstance(b, tuple) else b, current_torch_device(), False)


def get_worker_info():
    return torch.utils.data.get_worker_info()
