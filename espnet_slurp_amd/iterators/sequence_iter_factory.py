"""Per-epoch mini-batch iterator (espnet2/iterators/sequence_iter_factory.py:34-151) and the
data-parallel split of abs_task.build_sequence_iter_factory (abs_task.py:1520-1552).

Epoch e's batch order: the sampler's list shuffled by np.random.RandomState(e + seed) when
shuffling; with num_iters_per_epoch the epochs are cut from the concatenation of successive
shuffled passes exactly as the reference does (so a resumed run sees the same batches).
`shard_batches` gives rank r the keys batch[r::world] of every batch (min_batch_size =
world_size upstream).  `DevicePrefetcher` moves the next batch to the GPU on a side HIP
stream while the current step runs: the collate writes into page-locked buffers, so each
tensor is one async DMA, and the consumer stream waits on an event, never on the host.
"""
import random
from functools import partial
from typing import Any, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader


def worker_init_fn(worker_id, base_seed=0):
    seed = base_seed + worker_id
    random.seed(seed)
    np.random.seed(seed)


class RawSampler:
    def __init__(self, batches):
        self.batches = batches

    def __len__(self):
        return len(self.batches)

    def __iter__(self):
        return iter(self.batches)

    def generate(self, seed):
        return list(self.batches)


def shard_batches(batches: Sequence[Tuple[str, ...]], rank: int, world_size: int) -> List[Tuple[str, ...]]:
    for b in batches:
        if len(b) < world_size:
            raise RuntimeError(f"The batch-size must be equal or more than world_size: {len(b)} < {world_size}")
    return [tuple(b[rank::world_size]) for b in batches]


class SequenceIterFactory:
    def __init__(self, dataset, batches, num_iters_per_epoch: Optional[int] = None, seed: int = 0,
                 shuffle: bool = False, num_workers: int = 0, collate_fn=None, pin_memory: bool = False):
        self.sampler = batches if hasattr(batches, "generate") else RawSampler(batches)
        self.dataset = dataset
        self.num_iters_per_epoch = num_iters_per_epoch
        self.shuffle = shuffle
        self.seed = seed
        self.num_workers = num_workers
        self.collate_fn = collate_fn
        self.pin_memory = pin_memory

    def _pass(self, e: int, shuffle: bool) -> list:
        """The full (shuffled) batch list of pass e."""
        b = self.sampler.generate(e + self.seed)
        if shuffle:
            np.random.RandomState(e + self.seed).shuffle(b)
        return b

    def epoch_batches(self, epoch: int, shuffle: Optional[bool] = None) -> list:
        shuffle = self.shuffle if shuffle is None else shuffle
        n_it = self.num_iters_per_epoch
        if n_it is None:
            return self._pass(epoch, shuffle)
        N = len(self.sampler)
        if n_it < N:
            # window [n_it*(epoch-1), n_it*epoch) of the stream of passes 0, 1, 2, ...; the
            # reference indexes pass p by the integer quotient, its tail by the remainder
            p, off = divmod(n_it * epoch, N)
            if off >= n_it:
                return self._pass(p, shuffle)[off - n_it:off]
            return self._pass(p - 1, shuffle)[off - n_it:] + self._pass(p, shuffle)[:off]
        p, cur = divmod(n_it * (epoch - 1), N)
        need, out = n_it, []
        passes = self._pass(p, shuffle)
        while need > 0:
            take = passes[cur:cur + need]
            out += take
            if cur + need >= N:
                p, cur = p + 1, 0
                passes = self._pass(p, shuffle)
            else:
                cur += need
            need -= len(take)
        assert len(out) == n_it
        return out

    def build_iter(self, epoch: int, shuffle: Optional[bool] = None) -> DataLoader:
        kw = dict(collate_fn=self.collate_fn) if self.collate_fn is not None else {}
        return DataLoader(dataset=self.dataset, batch_sampler=self.epoch_batches(epoch, shuffle),
                          num_workers=self.num_workers, pin_memory=self.pin_memory,
                          worker_init_fn=partial(worker_init_fn, base_seed=epoch + self.seed), **kw)


class DevicePrefetcher:
    """Wrap an iterator of (utt_ids, {name: host tensor}) so that batch k+1's host->device
    copies run on a side stream during step k.  Lengths stay on the host (the model's host
    prep reads them without a device sync); float / token tensors go to `device`."""

    HOST_KEYS = ("_lengths",)

    def __init__(self, it, device, host_keys: Sequence[str] = HOST_KEYS):
        self.it = iter(it)
        self.device = torch.device(device)
        self.host_keys = tuple(host_keys)
        self.stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        self._next = None
        self._event = None
        self._preload()

    def _to_dev(self, k, v: torch.Tensor):
        if any(k.endswith(h) for h in self.host_keys) or k == "text":
            return v  # consumed on the host (lengths) or rewritten in place by the model (text)
        return v.to(self.device, non_blocking=True)

    def _preload(self):
        try:
            ids, batch = next(self.it)
        except StopIteration:
            self._next = None
            return
        if self.stream is None:
            self._next = (ids, {k: self._to_dev(k, v) for k, v in batch.items()})
            return
        with torch.cuda.stream(self.stream):
            moved = {k: self._to_dev(k, v) for k, v in batch.items()}
            self._event = torch.cuda.Event()
            self._event.record(self.stream)
        self._next = (ids, moved)

    def __iter__(self) -> Iterator[Tuple[List[str], dict]]:
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        cur, ev = self._next, self._event
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            for v in cur[1].values():  # the caching allocator must not recycle them early
                if v.is_cuda:
                    v.record_stream(torch.cuda.current_stream(self.device))
        self._preload()
        return cur
