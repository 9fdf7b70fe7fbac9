"""Fused Adam over the flat parameter buffer — the `adam` choice of espnet2
(abs_task.py:78-79 -> torch.optim.Adam) as one HIP kernel per step, applied after the
device-side clip_grad_norm_ (trainer.py:642-686).  Non-finite gradient norm => the kernel
skips the update (trainer.py:651-667) without a host round trip."""
from __future__ import annotations

import torch

from .. import kernels as K
from ..flat import FlatParams


def clip_grad_norm_(flat: FlatParams, max_norm: float, out: torch.Tensor = None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ on the flat gradient, on device.  Returns a 3-vector
    (total L2 norm, clip coefficient min(1, max_norm/(norm+1e-6)), finite flag); the
    coefficient is applied inside the Adam kernel."""
    if out is None:
        out = torch.empty(3, dtype=torch.float32, device=flat.grad.device)
    if flat.grad.is_cuda:
        K.join_side(flat.grad.device)
    K.grad_norm(flat.grad, max_norm, out)
    return out


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False):
        if amsgrad:
            raise NotImplementedError("amsgrad")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) != 1:
            raise NotImplementedError("FusedAdam: one param group (the espnet2 default)")
        self.flat = flat
        self.exp_avg = torch.zeros_like(flat.flat)
        self.exp_avg_sq = torch.zeros_like(flat.flat)
        self.n_steps = 0
        self._ones = torch.tensor([1.0, 1.0, 1.0], device=flat.flat.device)

    @torch.no_grad()
    def step(self, closure=None, clip: torch.Tensor = None):
        """clip: the 3-vector of clip_grad_norm_ (coefficient + finite flag); None = no clipping."""
        g = self.param_groups[0]
        self.n_steps += 1
        b1, b2 = g["betas"]
        K.adam(self.flat.flat, self.flat.grad, self.exp_avg, self.exp_avg_sq, clip if clip is not None else self._ones,
               g["lr"], b1, b2, g["eps"], g["weight_decay"], self.n_steps)
        return None

    # ---------------------------------------------------------- device-resident bookkeeping
    def device_state(self, scheduler=None) -> torch.Tensor:
        """{Adam steps applied, scheduler steps taken} as a device float64 pair, initialised from
        the host counters (graph mode keeps counting on device, esp_opt_advance)."""
        if getattr(self, "_dstate", None) is None:
            dev = self.flat.flat.device
            last = float(scheduler.last_epoch) if scheduler is not None else 0.0
            self._dstate = torch.tensor([float(self.n_steps), last], dtype=torch.float64, device=dev)
            self._hyper = torch.empty(3, dtype=torch.float32, device=dev)
        return self._dstate

    def step_device(self, clip: torch.Tensor, scheduler=None):
        """Adam step whose lr / bias corrections come from the device state (WarmupLR formula
        on device): capturable in a HIP graph.  Counts the step (and the scheduler step) on
        device only when the gradient norm was finite."""
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        st = self.device_state(scheduler)
        warmup = float(getattr(scheduler, "warmup_steps", 0.0) or 0.0)
        base = scheduler.base_lrs[0] if scheduler is not None else g["lr"]
        K.opt_hyper(st, base, warmup, b1, b2, self._hyper)
        K.adam_dev(self.flat.flat, self.flat.grad, self.exp_avg, self.exp_avg_sq, clip, self._hyper, b1, b2, g["eps"],
                   g["weight_decay"])
        K.opt_advance(st, clip)

    def sync_from_device(self, scheduler=None):
        """Copy the device counters back to the host objects (after graph replays)."""
        if getattr(self, "_dstate", None) is None:
            return
        n, s = (int(x) for x in self._dstate.tolist())
        self.n_steps = n
        if scheduler is not None and s != scheduler.last_epoch:
            scheduler.last_epoch = s
            for grp, lr in zip(self.param_groups, scheduler.get_lr()):
                grp["lr"] = lr

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def state_dict(self):
        sd = super().state_dict()
        sd["flat_state"] = {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self.n_steps}
        return sd
