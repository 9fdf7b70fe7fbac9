"""WarmupLR — espnet2/schedulers/warmup_lr.py:11-50:
lr = base_lr * warmup^0.5 * min(step^-0.5, step * warmup^-1.5), stepped per batch."""
from __future__ import annotations

from typing import Union

import torch
from torch.optim.lr_scheduler import _LRScheduler


class AbsScheduler:
    """abs_scheduler.py:6-19 (marker base)."""


class AbsBatchStepScheduler(AbsScheduler):
    """abs_scheduler.py:21-33: stepped after every optimizer step."""


class AbsEpochStepScheduler(AbsScheduler):
    """abs_scheduler.py:35-47: stepped once per epoch (Trainer.run)."""


class AbsValEpochStepScheduler(AbsEpochStepScheduler):
    """abs_scheduler.py:49-61: stepped once per epoch with the validation criterion value."""


class WarmupLR(_LRScheduler, AbsBatchStepScheduler):
    def __init__(self, optimizer: torch.optim.Optimizer, warmup_steps: Union[int, float] = 25000, last_epoch: int = -1):
        self.warmup_steps = warmup_steps
        super().__init__(optimizer, last_epoch)

    def __repr__(self):
        return f"{self.__class__.__name__}(warmup_steps={self.warmup_steps})"

    def lr_at(self, last_epoch: int):
        """The learning rates get_lr() gives once the scheduler's last_epoch is `last_epoch`
        (Trainer.train_one_epoch reconstructs the per-step lr it reports from this)."""
        step_num = last_epoch + 1
        return [lr * self.warmup_steps ** 0.5 * min(step_num ** -0.5, step_num * self.warmup_steps ** -1.5)
                for lr in self.base_lrs]

    def get_lr(self):
        step_num = self.last_epoch + 1
        return [lr * self.warmup_steps ** 0.5 * min(step_num ** -0.5, step_num * self.warmup_steps ** -1.5)
                for lr in self.base_lrs]
