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
            clip_grad_norm_(model.flat, opts.grad_clip, self._clip)
            self.optimizer.step(clip=self._clip)
            finite = True
            if check_finite:
                finite = bool(self._clip[2].item() != 0.0)
            if finite:
                if isinstance(self.scheduler, AbsBatchStepScheduler):
                    self.scheduler.step()
            else:
                self.n_skipped += 1
            self.optimizer.zero_grad()
        stats["grad_norm"] = self._clip[0:1]
        return stats

    def train_one_epoch(self, iterator: Iterable, reporter=None) -> bool:
        """Loop over (utt_id, batch) like trainer.py:502-714; returns True if every step was
        skipped (all_steps_are_invalid)."""
        self.model.train()
        all_invalid = True
        for _, batch in iterator:
            stats = self.train_one_step(batch)
            if reporter is not None:
                reporter(stats)
            all_invalid = all_invalid and (self.n_skipped == self.iiter)
        return all_invalid
