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

    # ---------------------------------------------------------- checkpoint interop
    def _adam_group(self) -> dict:
        """param_groups[0] as torch.optim.Adam would hold it (every Adam default key of this
        torch version, with this optimizer's hyper-parameters)."""
        g = self.param_groups[0]
        ref = torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))], lr=g["lr"], betas=g["betas"], eps=g["eps"],
                               weight_decay=g["weight_decay"])
        return dict(ref.param_groups[0])

    def state_dict(self):
        """torch.optim.Adam.state_dict() format — what the reference's checkpoint.pth holds under
        "optimizers" (trainer.py:340-352, abs_task.py:78-79): per parameter (keyed by its index
        in param_groups[0]["params"]) {"step": float32 scalar, "exp_avg", "exp_avg_sq"} with the
        parameter's shape, copied out of the flat moment buffers.  Graph mode keeps the step
        count on device: it is read from there.  The group's lr is the host value — call
        Trainer.sync_host_state() first (train_one_epoch does)."""
        g = self.param_groups[0]
        n = int(self._dstate[0].item()) if getattr(self, "_dstate", None) is not None else self.n_steps
        state = {}
        if n > 0:
            for i, p in enumerate(g["params"]):
                o, k = self.flat.slots[id(p)]
                state[i] = {"step": torch.tensor(float(n), dtype=torch.float32),
                            "exp_avg": self.exp_avg[o:o + k].view(p.shape).clone(),
                            "exp_avg_sq": self.exp_avg_sq[o:o + k].view(p.shape).clone()}
        group = self._adam_group()
        group["params"] = list(range(len(g["params"])))
        if "initial_lr" in g:  # added by the LR scheduler (torch _LRScheduler.__init__)
            group["initial_lr"] = g["initial_lr"]
        return {"state": state, "param_groups": [group]}

    @torch.no_grad()
    def load_state_dict(self, state_dict):
        """Load a torch.optim.Adam state_dict (the reference's checkpoint, or ours): the moments
        are copied into the flat buffers in place (a captured HIP graph keeps pointing at them),
        the step count into the host and device counters.  FusedAdam keeps ONE step count: a
        checkpoint whose parameters have different Adam step counts is refused."""
        saved_groups = state_dict["param_groups"]
        g = self.param_groups[0]
        if len(saved_groups) != 1 or len(saved_groups[0]["params"]) != len(g["params"]):
            raise ValueError("loaded state dict has a different number of parameter groups / parameters")
        sg = saved_groups[0]
        if sg.get("amsgrad", False):
            raise NotImplementedError("amsgrad")
        for key in ("lr", "betas", "eps", "weight_decay"):
            g[key] = tuple(sg[key]) if key == "betas" else sg[key]
        if "initial_lr" in sg:  # set by the LR scheduler at construction
            g["initial_lr"] = sg["initial_lr"]
        index = dict(zip(sg["params"], g["params"]))
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        steps = set()
        for i, st in state_dict["state"].items():
            p = index[int(i)]
            o, k = self.flat.slots[id(p)]
            if st["exp_avg"].numel() != k:
                raise ValueError(f"state of parameter {i}: {tuple(st['exp_avg'].shape)} != {tuple(p.shape)}")
            self.exp_avg[o:o + k].copy_(st["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
            steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError(f"parameters have different Adam step counts {sorted(steps)}")
        self.n_steps = steps.pop() if steps else 0
        if getattr(self, "_dstate", None) is not None:
            self._dstate[0].fill_(float(self.n_steps))

    def refresh_device_state(self, scheduler=None):
        """After loading optimizer / scheduler state: write the host counters into the device
        state in place (graph mode reads the lr schedule position from there)."""
        if getattr(self, "_dstate", None) is None:
            return
        last = float(scheduler.last_epoch) if scheduler is not None else 0.0
        self._dstate.copy_(torch.tensor([float(self.n_steps), last], dtype=torch.float64))
