"""Data-parallel gradient exchange over RCCL (torch.distributed 'nccl' == RCCL on ROCm).

Replaces DDP's bucketed all-reduce (trainer.py:214-236, X6 of SURVEY.md §2.2) with buckets
cut from the flat gradient buffer (flat.py) in backward-completion order: as the explicit
backward finishes a module (decoder layer, encoder block, ...) the module's slice is marked
ready; a bucket whose slice is complete is all-reduced asynchronously, overlapping the
remaining backward kernels (RCCL orders itself after the work already on the stream).
Gradients are averaged as SUM + a 1/world scale on device, on every backend (round 6: RCCL's
ReduceOp.AVG had only ever run at world 1, while the world-2 tests took the gloo SUM branch -- now the
tested code IS the RCCL code; for world a power of two the scale is exact, so the result is DDP's
average bit for bit given the same summation order).
The per-step scalar statistics (X4/X5) travel in one small fused all-reduce.
BatchNorm statistics stay per-replica (no SyncBN), as in the reference; rank 0's BN
buffers are broadcast at each forward when `broadcast_buffers` (DDP default, X7).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.distributed as dist

from .. import kernels as K
from ..flat import FlatParams


class FlatGradReducer:
    def __init__(self, model, flat: FlatParams, bucket_mb: float = 25.0, group=None, hooks: bool = True):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.bucket_elems = int(bucket_mb * (1 << 20) / 4)
        # buckets over [0, numel) cut at parameter boundaries, from the END (first ready)
        offs = sorted(flat.slots[id(p)] for _, p in flat.params)
        bounds: List[Tuple[int, int]] = []
        end = flat.numel
        start = end
        for o, n in reversed(offs):
            start = o
            if end - start >= self.bucket_elems:
                bounds.append((start, end))
                end = start
        if end > 0:
            bounds.append((0, end))
        self.buckets = bounds  # in launch order
        self.param_bucket: Dict[int, int] = {}
        self.bucket_count = [0] * len(bounds)
        for _, p in flat.params:
            o, _n = flat.slots[id(p)]
            for bi, (s, e) in enumerate(bounds):
                if s <= o < e:
                    self.param_bucket[id(p)] = bi
                    self.bucket_count[bi] += 1
                    break
        self._reset()
        if hooks:  # eager mode: launch buckets as the explicit backward completes modules
            model._grad_hook = self.module_done
            for m in (getattr(model, "encoder", None), getattr(model, "decoder", None)):
                if m is not None:
                    m._grad_hook = self.module_done

    sync = True  # False between the micro-batches of one optimizer step (DDP.no_sync)

    def _reset(self):
        self.ready = [0] * len(self.buckets)
        self.seen = set()
        self.handles = {}
        self.next_launch = 0

    def _launch_ready(self):
        # launch in order so every rank issues the same collective sequence
        while self.next_launch < len(self.buckets) and self.ready[self.next_launch] == self.bucket_count[self.next_launch]:
            s, e = self.buckets[self.next_launch]
            t = self.flat.grad[s:e]
            self.handles[self.next_launch] = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self.next_launch += 1

    def module_done(self, module):
        if not self.sync:  # an earlier micro-batch of accum_grad: accumulate locally
            return
        for p in module.parameters():
            if id(p) in self.seen or id(p) not in self.param_bucket:
                continue
            self.seen.add(id(p))
            self.ready[self.param_bucket[id(p)]] += 1
        self._launch_ready()

    def finish(self):
        """Launch whatever is left, wait for every bucket; grads are the replica average."""
        for bi in range(len(self.buckets)):
            self.ready[bi] = self.bucket_count[bi]
        self._launch_ready()
        for h in self.handles.values():
            h.wait()
        # the average: the same SUM + scale whatever the backend (the world-2 gloo tests run this code)
        if self.world == 1:
            pass
        elif self.flat.grad.is_cuda:
            K.scale_dropout(self.flat.grad, self.flat.grad, alpha=1.0 / self.world)
        else:  # host tensors (the CPU multi-process tests)
            self.flat.grad.mul_(1.0 / self.world)
        self._reset()

    def allreduce_sum(self):
        """SUM all-reduce of the whole flat gradient in the same buckets (HIP-graph mode: the
        caller pre-scaled each replica's gradient by w_r / sum w)."""
        hs = [dist.all_reduce(self.flat.grad[s:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
              for s, e in self.buckets]
        for h in hs:
            h.wait()

    def launch_sum(self, bucket_ids):
        """Asynchronous SUM all-reduces of the given buckets (the HIP-graph path, whose replicas
        pre-scaled their gradients by w_r / sum w); returns the work handles."""
        return [dist.all_reduce(self.flat.grad[self.buckets[b][0]:self.buckets[b][1]], op=dist.ReduceOp.SUM,
                                group=self.group, async_op=True) for b in bucket_ids]

    def plan_hook(self, on_ready):
        """A module-done hook that launches nothing: it tracks bucket readiness like
        module_done and calls on_ready(bucket_ids) whenever the in-order launch front advances
        (used while capturing the backward in segments, one segment per launch point)."""
        ready = [0] * len(self.buckets)
        seen = set()
        front = [0]

        def hook(module):
            for p in module.parameters():
                if id(p) in seen or id(p) not in self.param_bucket:
                    continue
                seen.add(id(p))
                ready[self.param_bucket[id(p)]] += 1
            ids = []
            while front[0] < len(self.buckets) and ready[front[0]] == self.bucket_count[front[0]]:
                ids.append(front[0])
                front[0] += 1
            if ids:
                on_ready(ids)

        def rest():
            ids = list(range(front[0], len(self.buckets)))
            front[0] = len(self.buckets)
            return ids

        hook.rest = rest
        hook.done = lambda: front[0] >= len(self.buckets)
        return hook

    def broadcast_buffers(self, model, async_op: bool = False):
        """DDP's broadcast_buffers (X7): rank 0's floating buffers (BatchNorm running stats) to
        every replica before the forward, as ONE broadcast of the flat buffer they are views
        of (flat.py).  Training-mode outputs do not read them, so this only keeps the
        replicas' eval-mode state equal to rank 0's.  async_op: returns the work handles."""
        hs = []
        if self.flat.buffers:
            hs.append(dist.broadcast(self.flat.buf_flat, 0, group=self.group, async_op=async_op))
        for b in self.flat.other_buffers:
            hs.append(dist.broadcast(b, 0, group=self.group, async_op=async_op))
        return [h for h in hs if h is not None] if async_op else []


def fused_stats_allreduce(stats: Dict[str, torch.Tensor], weight: torch.Tensor, group=None):
    """recursive_average (espnet2/torch_utils/recursive_op.py:8-47) in ONE all-reduce:
    returns (weighted-average stats, summed weight) as device tensors (no host sync)."""
    keys = [k for k, v in stats.items() if v is not None]
    w = weight.to(torch.float32).view(1)
    vec = torch.cat([stats[k].view(-1)[:1].float() * w for k in keys] + [w])
    dist.all_reduce(vec, group=group)
    tot = vec[-1:]
    return {k: vec[i:i + 1] / tot for i, k in enumerate(keys)}, tot
