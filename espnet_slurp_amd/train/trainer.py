"""Trainer step — the hot loop of espnet2/train/trainer.py:463-720 (train_one_epoch).

Per batch: forward (model(**batch)), weighted loss normalisation (:594-608), backward,
bucketed RCCL gradient average (replaces DDP), clip_grad_norm_(grad_clip) on device,
non-finite skip (:651-667), Adam + WarmupLR batch step (:671-686), zero_grad.
Host synchronisation: one 3-float read (grad norm / finite flag) per optimizer step, which
the reference also needs (torch.isfinite(grad_norm) on the host, :651).
"""
from __future__ import annotations

import dataclasses
import time
from typing import Dict, Iterable, Optional

import torch
import torch.distributed as dist

from ..optimizers.fused_adam import FusedAdam, clip_grad_norm_
from ..schedulers.warmup_lr import AbsBatchStepScheduler
from .distributed import FlatGradReducer, fused_stats_allreduce


@dataclasses.dataclass
class TrainerOptions:
    grad_clip: float = 5.0
    grad_clip_type: float = 2.0
    accum_grad: int = 1
    no_forward_run: bool = False
    log_interval: Optional[int] = None


class Trainer:
    def __init__(self, model, optimizer: FusedAdam, scheduler=None, options: TrainerOptions = None,
                 distributed: bool = False, bucket_mb: float = 25.0):
        self.model = model
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.options = options or TrainerOptions()
        self.distributed = distributed and dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size() if self.distributed else 1
        self.reducer = FlatGradReducer(model, model.flat, bucket_mb) if self.distributed else None
        self.iiter = 0
        self.n_skipped = 0
        self._clip = torch.empty(3, dtype=torch.float32, device=model.flat.flat.device)
        # finite flag of the last optimizer step, read back asynchronously (pinned buffer + event)
        # and acted on just before the NEXT optimizer step: the host never drains the queue
        cuda = self._clip.is_cuda
        self._flag_host = torch.empty(1, dtype=torch.float32, pin_memory=cuda)
        self._flag_event = torch.cuda.Event() if cuda else None
        self._pending = False

    def train_one_step(self, batch: Dict[str, torch.Tensor], check_finite: bool = True) -> Dict[str, torch.Tensor]:
        """One iteration of train_one_epoch's loop body; returns device-side stats."""
        opts = self.options
        self.iiter += 1
        model = self.model
        if self.distributed and self.reducer is not None:
            pass
        loss, stats, weight = model(**batch)
        stats = {k: v for k, v in stats.items() if v is not None}
        if self.distributed:
            w = weight.to(torch.float32).view(1)
            stats, wsum = fused_stats_allreduce(stats, weight)
            # (loss*weight).sum()/sum(weight)*world_size, DDP then averages  (trainer.py:594-606)
            loss = (loss * w).sum() / wsum * self.world
        loss = loss / opts.accum_grad
        loss.backward()
        if self.iiter % opts.accum_grad == 0:
            if self.reducer is not None:
                self.reducer.finish()
            self.resolve_pending()  # scheduler step of the previous update (if it was finite)
            clip_grad_norm_(model.flat, opts.grad_clip, self._clip)
            # the Adam kernel itself skips a non-finite update on device (trainer.py:651-667)
            self.optimizer.step(clip=self._clip)
            if check_finite:
                self._flag_host.copy_(self._clip[2:3], non_blocking=True)
                if self._flag_event is not None:
                    self._flag_event.record()
                self._pending = True
            elif isinstance(self.scheduler, AbsBatchStepScheduler):
                self.scheduler.step()
            self.optimizer.zero_grad()
        stats["grad_norm"] = self._clip[0:1]
        return stats

    def resolve_pending(self):
        """Apply the bookkeeping of the last optimizer step once its finite flag is on the host:
        WarmupLR batch step if the gradient norm was finite, else count a skipped step
        (trainer.py:651-686).  Called before the next optimizer step and at epoch end."""
        if not self._pending:
            return
        if self._flag_event is not None:
            self._flag_event.synchronize()
        self._pending = False
        if float(self._flag_host[0]) != 0.0:
            if isinstance(self.scheduler, AbsBatchStepScheduler):
                self.scheduler.step()
        else:
            self.n_skipped += 1

    def train_one_epoch(self, iterator: Iterable, reporter=None) -> bool:
        """Loop over (utt_id, batch) like trainer.py:502-714; returns True if every step was
        skipped (all_steps_are_invalid)."""
        self.model.train()
        it0, sk0 = self.iiter, self.n_skipped
        for _, batch in iterator:
            stats = self.train_one_step(batch)
            if reporter is not None:
                reporter(stats)
        self.resolve_pending()
        return (self.n_skipped - sk0) == (self.iiter - it0)
